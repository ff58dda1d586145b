#!/bin/bash
# Alternating A/B of whole bench runs: this tree, a copy of an earlier commit under ab_old/ (its own
# library and ext built there), and this tree's Python over ab_old's library.  BENCH_ARGS: bench flags.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
A=${BENCH_ARGS:---no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --steps 100}
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $A > $OUT/ab_new.$rep.json 2> $OUT/ab_new.$rep.err || { tail $OUT/ab_new.$rep.err; exit 1; }
  timeout -k 10 200 python ab_old/bench.py $A > $OUT/ab_old.$rep.json 2> $OUT/ab_old.$rep.err || { tail $OUT/ab_old.$rep.err; exit 1; }
  GSRAST_LIB=$R/ab_old/gaussian-splatting-skysphere_amd/build/libgsrast.so timeout -k 10 200 python bench.py $A > $OUT/ab_oldlib.$rep.json 2> $OUT/ab_oldlib.$rep.err || { tail $OUT/ab_oldlib.$rep.err; exit 1; }
  for v in new old oldlib; do
    python -c "
import json; d = json.load(open('$OUT/ab_$v.$rep.json'))
print('%-7s value %8.1f  sustained %8.1f  serial_one_stream %8.1f' % ('$v', d['value'], d['sustained']['iters_s'], d['serial_one_stream']['iters_s']))"
  done
done
