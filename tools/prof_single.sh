#!/bin/bash
# rocprofv3 kernel trace + stats of the batch-1 loop (tools/prof_single.py); optional PMC passes over
# render_bwd's SQ counters.  Each GPU step has its own limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_single -o run --output-format csv -- python3 $R/tools/prof_single.py --steps ${STEPS:-20} > $OUT/prof_single.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_single.log; exit 1; }
cd $R
python3 tools/kstats.py $OUT/prof_single $(( ${STEPS:-20} + 3 ))
echo done
