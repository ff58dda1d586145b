#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
SV_ARGS="--steps 60" timeout -k 10 300 bash tools/sv_ab.sh build_r4 build_p768 build_p1536 > $OUT/r05_sv_occ.txt 2>&1 || { cat $OUT/r05_sv_occ.txt; exit 1; }
cat $OUT/r05_sv_occ.txt
