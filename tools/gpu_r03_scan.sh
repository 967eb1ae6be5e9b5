# Round 3: radix scan with register-held runs -- Lovasz parity (incl. a 1M-pixel image), lib A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_losses_full.py tests/test_gpu_ops.py tests/test_gpu_round2.py tests/test_gpu_targets.py tests/test_gpu_determinism.py -k "lovasz or Lovasz or loss or golden or determinism or ignore" > gpurun_out/scan_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/scan_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/scan_t.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scan_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/scan_prof.log 2>&1 || { echo prof failed; exit 1; }
grep -i "radix\|lovasz" gpurun_out/scan_prof/run_kernel_stats.csv | cut -c1-160
echo done
