#!/bin/bash
# Builds the CPU oracle with 32x32 binning tiles (a copy under /tmp; the repo's oracle is untouched)
# and runs tools/supertile_stats.py on the C3 scene (CPU only, ~30 s on 8 cores).
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
D=${TMPDIR:-/tmp}/gs_oracle_tile32
mkdir -p $D
sed -e 's/^#define TILE 16$/#define TILE 32/' -e 's/16\.0f/((float)TILE)/g' \
    -e 's/(X0 - 15\.0f)/(X0 - ((float)TILE - 1.0f))/' $R/oracle/gs_oracle.c > $D/gs_oracle.c
grep -q '^#define TILE 32$' $D/gs_oracle.c
gcc -O2 -fopenmp -fPIC -ffp-contract=off -fno-fast-math -std=c11 -shared -o $D/libgs_oracle.so $D/gs_oracle.c -lm -fopenmp
make -s -C $R/oracle
python $R/tools/supertile_stats.py $D/libgs_oracle.so
