#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit; stop at the first step that
# faults, aborts or times out (exit status other than 0 / 1: a failing test or assertion is 1 and the
# next step still runs).  Usage (from the repo root, via gpurun):
#   tools/gpu_steps.sh OUTDIR "SECONDS:NAME:COMMAND" ["SECONDS:NAME:COMMAND" ...]
# Each step's stdout+stderr go to OUTDIR/NAME.log; a summary line per step is printed.
set -u
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  secs=${spec%%:*}
  rest=${spec#*:}
  name=${rest%%:*}
  cmd=${rest#*:}
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n 3 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
