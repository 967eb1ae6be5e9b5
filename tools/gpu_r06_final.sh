# round-6 close: the whole -m gpu suite, smoke(), and the default bench line, one box
#   COMMIT=<sha> bash tools/gpu_r06_final.sh      (outputs under gpurun_out/r06_final_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r06_final_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || { tail -30 gpurun_out/r06_final_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final_smoke.log 2>&1 || { tail -20 gpurun_out/r06_final_smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.err || { tail -20 gpurun_out/r06_final_bench.err; exit 1; }
python - "${COMMIT:-unknown}" <<'PYEOF'
import json, sys
commit = sys.argv[1]
t = open("gpurun_out/r06_final_tests.log").read().strip().splitlines()
s = open("gpurun_out/r06_final_smoke.log").read().strip().splitlines()
with open("gpurun_out/r06_final_summary.txt", "w") as f:
    f.write(f"# commit {commit}: python -m pytest tests -m gpu; __graft_entry__.smoke(); python bench.py (defaults)\n")
    f.write(t[-1] + "\n" + s[-1] + "\n")
d = json.loads(open("gpurun_out/r06_final_bench.json").read().strip().splitlines()[-1])
d["commit"] = commit
open("gpurun_out/r06_final_bench.json", "w").write(json.dumps(d) + "\n")
print(d["value"], {k: v["value"] for k, v in (d.get("configs") or {}).items()})
PYEOF
cat gpurun_out/r06_final_summary.txt
