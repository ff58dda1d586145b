#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
exit $rc
