# SQ stall / instruction / L2 hit counters of the conv kernels of one shape (SH; default the big 3x3
# decoder ring shape), one rocprofv3 pass per counter group
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SH=${SH:-16,32,32,1024,2048,512,3,1,1}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcring -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmcring.log 2>&1 || { echo PMC FAILED; tail -5 gpurun_out/pmcring.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcring2 -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmcring2.log 2>&1 || { echo PMC2 FAILED; tail -5 gpurun_out/pmcring2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcring3 -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmcring3.log 2>&1 || { echo PMC3 FAILED; tail -5 gpurun_out/pmcring3.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmcring", "gpurun_out/pmcring2", "gpurun_out/pmcring3"):
    f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void (anonymous namespace)::", "")[:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        if "tn_fast" not in k and "wgrad" not in k and "halo" not in k:
            continue
        print(k)
        print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
PY
rm -rf gpurun_out/pmcring gpurun_out/pmcring2 gpurun_out/pmcring3
