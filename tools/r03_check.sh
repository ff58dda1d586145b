#!/bin/bash
# Round-3 GPU routine: gpu tests (one process, per-test timeout) then the default C3 bench without
# the CPU baseline.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench.log") if l.startswith("{")][0])
print("value", d["value"], "ms", d["ms_per_step"], "sustained", (d.get("sustained") or {}).get("iters_s"))
sv = d.get("single_view") or {}
print("single_view", sv.get("iters_s"), "ms", sv.get("ms_per_iter"), "kernel sum", sv.get("kernel_us_sum"))
for k, v in (sv.get("kernel_us_per_iter") or {}).items():
    print(f"  {k:18s} {v:8.2f} us")
print("train_step", (d.get("train_step") or {}).get("fused"))
PY
echo done
