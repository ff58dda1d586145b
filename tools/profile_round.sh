#!/bin/bash
# Round profile set: C3 bench with CPU baseline, rocprofv3 kernel stats of the bench command, PMC
# traffic / VALU passes, C5 + C2 bench lines.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -20 $OUT/bench_c3.log; exit 1; }
echo "bench c3 ok"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
echo "rocprof ok"
cd $R
bash tools/pmc_passes.sh > $OUT/pmc_passes.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc_passes.log; exit 1; }
python3 tools/pmc_traffic.py $OUT c3 $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1 || { echo "pmc_traffic failed"; exit 1; }
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1
echo "pmc ok"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload c5 > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -20 $OUT/bench_c5.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --workload c2 > $OUT/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.log; exit 1; }
echo done
