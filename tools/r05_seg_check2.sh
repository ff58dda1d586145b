#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 bash tools/sv_ab.sh build build_a build_r4 build_s256 > $OUT/r05_sv_ab2.txt 2>&1 || { cat $OUT/r05_sv_ab2.txt; exit 1; }
cat $OUT/r05_sv_ab2.txt
timeout -k 10 600 bash tools/r05_pmc_ab.sh build build_r4 > $OUT/r05_pmc_ab2.txt 2>&1 || { cat $OUT/r05_pmc_ab2.txt; exit 1; }
for b in build build_r4; do echo "== $b"; python3 tools/pmc_summary.py gpurun_out pmcab_${b}_; done
