#!/bin/bash
# A/B of the train step with and without the split-SH rasterizer inputs, in one GPU call:
# plain timing (alternating, 3 rounds each) and one rocprofv3 kernel trace of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for k in 1 2 3 4; do
  for m in "" "--no-split-sh"; do
    timeout -k 10 200 python tools/prof_train_step.py --steps 200 --warmup 10 $m > $OUT/ab_split$m.log 2>&1 || { echo "run $m failed"; tail $OUT/ab_split$m.log; exit 1; }
    echo "split${m:-=on} $(tail -1 $OUT/ab_split$m.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for m in "" "--no-split-sh"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/abprof$m -o run --output-format csv -- python3 $R/tools/prof_train_step.py --steps 30 --warmup 5 $m > $OUT/abprof$m.log 2>&1 || { echo "prof $m failed"; exit 1; }
  echo "prof split${m:-=on} $(grep 'train step' $OUT/abprof$m.log)"
done
