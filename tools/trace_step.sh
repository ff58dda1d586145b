#!/bin/bash
# rocprofv3 kernel trace of a few plain C3 steps (no HIP-event profiling) -> gpurun_out/trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/prof_step.py --workload ${WL:-c3} --steps 5 --warmup 3 > $OUT/trace.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/trace.log; exit 1; }
cd $R && python3 tools/timeline.py $OUT/trace/run_kernel_trace.csv
