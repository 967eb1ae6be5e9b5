# bitwise A/B of two library builds on C2 / C4 / C5 (tools/ab_bitwise.py), then the interleaved bench A/B
#   bash tools/gpu_ab_bitwise.sh <old lib dir>      (dumps under /tmp on the box; results on stdout)
set -o pipefail
OLD=$1
for cfg in "unet_resnet50 16" "attention_unet 8" "multitask_unet 8"; do
  set -- $cfg
  UNETSEG_LIB_PATH=$OLD/libunetseg_hip.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.pt $1 $2 2>/dev/null || exit 1
  timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.pt $1 $2 2>/dev/null || exit 1
  python tools/ab_bitwise.py compare /tmp/ab_a.pt /tmp/ab_b.pt
done
rm -f /tmp/ab_a.pt /tmp/ab_b.pt
NB=${NB:-2} EXTRA=1 bash tools/gpu_ab.sh UNETSEG_LIB_PATH=$OLD/libunetseg_hip.so -
