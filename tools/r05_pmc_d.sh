#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
KRE=render_bwd timeout -k 10 400 bash tools/r05_pmc_ab.sh build_d > $OUT/r05_pmc_d.txt 2>&1 || { cat $OUT/r05_pmc_d.txt; exit 1; }
python3 tools/pmc_summary.py gpurun_out pmcab_build_d_
