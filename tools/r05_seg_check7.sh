#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
SV_ARGS="--steps 60" timeout -k 10 300 bash tools/sv_ab.sh build build_r4 > $OUT/r05_sv_ab7.txt 2>&1 || { cat $OUT/r05_sv_ab7.txt; exit 1; }
cat $OUT/r05_sv_ab7.txt
TAG=steal2 timeout -k 10 300 bash tools/r05_timing.sh || exit 1
KRE=render_bwd timeout -k 10 400 bash tools/r05_pmc_ab.sh build > $OUT/r05_pmc_steal2.txt 2>&1 || { cat $OUT/r05_pmc_steal2.txt; exit 1; }
python3 tools/pmc_summary.py gpurun_out pmcab_build_
