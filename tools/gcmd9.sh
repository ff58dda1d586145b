set -o pipefail
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sv -o run --output-format csv -- python3 $R/tools/sv_ab.py --graph --no-prof --steps 30 > $OUT/prof_sv.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_sv.log; exit 1; }
cd $R
f=$(ls $OUT/prof_sv/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $OUT/prof_sv -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $f | tail -40
