#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 bash tools/sv_ab.sh build_d build_dnt build_dnt2 build_d256 build_dinf build_r4 > $OUT/r05_sv_ab3.txt 2>&1 || { cat $OUT/r05_sv_ab3.txt; exit 1; }
cat $OUT/r05_sv_ab3.txt
