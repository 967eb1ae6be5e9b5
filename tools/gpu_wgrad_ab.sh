# wgrad kernel durations (split-K kernel and reduce separately) of single conv shapes under several
# library environments: VARIANTS = ';'-separated env assignments, SHAPES = conv_bench shape list
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SHAPES=${SHAPES:-"16,32,32,1024,0,256,1,1,0 16,128,128,64,0,256,1,1,0 16,16,16,512,0,512,3,1,1 16,32,32,512,0,512,3,2,1 16,128,128,256,0,64,1,1,0 16,64,64,512,0,1024,1,2,0"}
IFS=';' read -ra VS <<< "${VARIANTS:-UNETSEG_WG_NO_RING=1;UNETSEG_WG_RING_NS=4;UNETSEG_WG_RING_NS=6;UNETSEG_WG_RING_NS=8}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  ( export $v; REPS=5 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wab$i -o run -- python tools/conv_bench.py $SHAPES > gpurun_out/wab$i.log 2>&1 ) || { echo "FAILED $v"; tail -20 gpurun_out/wab$i.log; exit 1; }
  echo "== $v"
  grep -v "^initialize\|amdgpu.ids" gpurun_out/wab$i.log | grep -v "^\[" | head -20
  python - "gpurun_out/wab$i" <<'PY'
import csv, glob, re, sys, collections
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0])))
agg = collections.OrderedDict()
for r in rows:
    k = r["Kernel_Name"]
    if not re.search("wgrad", k):
        continue
    key = (k.replace("void (anonymous namespace)::", "").split("(")[0][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, gx, gy, gz), v in agg.items():
    v = sorted(v)[: max(1, len(v) // 2)]
    print(f"  {min(v):8.1f} us  grid {gx}x{gy}x{gz:<6s} {k}")
PY
  rm -rf gpurun_out/wab$i
done
