set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SH=${SH:-16,512,512,64,0,64,3,1,1}
timeout -k 10 120 python3 tools/conv_bench.py $SH 16,256,256,64,0,64,3,1,1 16,128,128,64,0,64,3,1,1 2>&1 | grep -v amdgpu.ids
STATS=1 timeout -k 10 120 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids
SH=$SH timeout -k 10 400 bash tools/gpu_pmc_ring.sh
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmcf.log 2>&1 || { echo PMCF FAILED; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmcf/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("void (anonymous namespace)::", "")[:60]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k, "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
PY
rm -rf gpurun_out/pmcf
