cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/gputest.log; grep -E "^E  .*Error" gpurun_out/gputest.log | head -5
exit $rc
