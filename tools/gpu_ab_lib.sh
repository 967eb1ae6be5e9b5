# interleaved bench A/B of two library builds ($NB rounds): A = ${LIB_A:-tools/ab/A/libunetseg_hip.so}
# (`make -C unet-embroidery-seg_amd/csrc OUT=$PWD/tools/ab/A/libunetseg_hip.so` on the old sources builds
# the library AND its fast-call binding there), B = the in-tree build.  Both arms load their own
# fast-call binding (lib.py), so the A/B runs at the production host cost.
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in $(seq 1 ${NB:-3}); do
  for v in A B; do
    if [ $v = A ]; then L=${LIB_A:-tools/ab/A/libunetseg_hip.so}; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
    UNETSEG_LIB_PATH=$L timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['ms_per_step'])" || exit 1
  done
done
