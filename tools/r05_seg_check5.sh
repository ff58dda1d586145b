#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
SV_ARGS="--steps 60" timeout -k 10 500 bash tools/sv_ab.sh build build_s64 build_s256 build_tf build_r4 > $OUT/r05_sv_ab5.txt 2>&1 || { cat $OUT/r05_sv_ab5.txt; exit 1; }
cat $OUT/r05_sv_ab5.txt
TAG=e4 timeout -k 10 300 bash tools/r05_timing.sh
