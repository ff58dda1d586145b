#!/bin/bash
# GPU-box routine: parity tests, bench, rocprofv3 kernel-trace summary.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
if [ -n "$PROFILE" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
fi
if [ -n "$PMC" ]; then
  cd /tmp
  for pass in fetch:FETCH_SIZE write:WRITE_SIZE sq2:SQ_INSTS_VALU; do
    name=${pass%%:*}; ctr=${pass#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/pmc_$name -o run --output-format csv -- python3 $R/tools/prof_step.py --workload c3 --steps 2 --warmup 1 > $OUT/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -20 $OUT/pmc_$name.log; exit 1; }
  done
  cd $R
  python tools/pmc_traffic.py $OUT c3 $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1 || { echo "pmc_traffic failed"; exit 1; }
fi
echo done
