#!/bin/bash
# repeatability of the default bench line (the driver's command) against a run without the
# post-timing legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() {
  timeout -k 10 400 python bench.py "$@" > $OUT/dc.log 2>&1 || { tail $OUT/dc.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/dc.log') if l.startswith('{')][0]); print('$*', 'value', d['value'], 'sustained', (d.get('sustained') or {}).get('iters_s'))"
}
run
run --no-cpu-baseline --no-train-step
run
run --no-cpu-baseline --no-train-step
run --steps 400
