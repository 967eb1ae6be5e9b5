# Round-5 end-of-round record, part 1: the whole -m gpu suite (with the teacher reports written to
# gpurun_out/r05_teacher/) and smoke, on one box.  COMMIT (the tree's sha, substituted on the host)
# heads the summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_teacher
UNETSEG_TEACHER_OUT=gpurun_out/r05_teacher timeout -k 10 1050 python -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/r05_gputest.log 2>&1
rc=$?
{ echo "# commit ${COMMIT:-unknown}"; echo "# python -m pytest tests -m gpu -q (exit $rc)"; tail -4 gpurun_out/r05_gputest.log; } > gpurun_out/r05_gputest_summary.txt
[ $rc -eq 0 ] || { tail -30 gpurun_out/r05_gputest.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r05_gputest_summary.txt 2>&1
cat gpurun_out/r05_gputest_summary.txt
