#!/bin/bash
# timed-region sensitivity to warm-up length (C3, short timed regions)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for w in 5 5 5 50 50 50; do
  timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-train-step --sustain-s 0 > $OUT/warm.log 2>&1 || { tail $OUT/warm.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/warm.log') if l.startswith('{')][0]); print('warmup', $w, 'value', d['value'], 'ms/step', d['ms_per_step'])"
done
