#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
SV_ARGS="--steps 60" timeout -k 10 300 bash tools/sv_ab.sh build build_pad build_r4 > $OUT/r05_sv_pad.txt 2>&1 || { cat $OUT/r05_sv_pad.txt; exit 1; }
cat $OUT/r05_sv_pad.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05_gpu_tests_v3.txt 2>&1; rc=$?
tail -5 $OUT/r05_gpu_tests_v3.txt
exit $rc
