#!/bin/bash
# Round 5: segmented backward -- batch-1 A/B against round 4's library, per-wave stamps, GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 bash tools/sv_ab.sh build build_r4 build_s64 build_s256 > $OUT/r05_sv_ab1.txt 2>&1 || { cat $OUT/r05_sv_ab1.txt; exit 1; }
cat $OUT/r05_sv_ab1.txt
GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/build_timing/libgsrast.so timeout -k 10 200 python -u tools/bwd_timing.py --workload c3 --reps 2 --out $OUT/r05_bwd_timing_c3_v1.json > $OUT/r05_bwd_timing_c3_v1.log 2>&1 || { tail $OUT/r05_bwd_timing_c3_v1.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05_gpu_tests_v1.txt 2>&1; rc=$?
tail -15 $OUT/r05_gpu_tests_v1.txt
exit $rc
