#!/bin/bash
# GPU test run: pytest -m gpu (one process, per-test timeout), log under gpurun_out/
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 ${GS_TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gputest.log
tail -5 gpurun_out/gputest.log
exit $rc
