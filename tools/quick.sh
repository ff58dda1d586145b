#!/bin/bash
# Quick GPU iteration: gpu parity tests + C3 bench (no CPU baseline).  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench.log") if l.startswith("{")][0])
print("value", d["value"], "ms", d["ms_per_step"], "render_mpix_s", d["render_mpix_s"])
for k, v in d["kernels"].items():
    print(f"  {k:16s} {v['total_ms_per_step']:.4f} ms  x{v['launches_per_step']}  avg {v['avg_us']} us")
PY
