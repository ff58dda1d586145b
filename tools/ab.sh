#!/bin/bash
# A/B two library builds on the bench (same process settings, sequential runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for b in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$b/libgsrast.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/ab_$b.log 2>&1 || { echo "bench $b failed"; tail $OUT/ab_$b.log; exit 1; }
done
echo ab done
