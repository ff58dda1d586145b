# kernel timeline of the fused-Adam train step with the per-iteration loss.item() (rocprofv3 kernel
# trace only), and without the fused Adam for comparison
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
for m in "--fuse-adam" ""; do
  tag=$( [ -n "$m" ] && echo fa || echo unf )
  timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/ts_trace_$tag -o run --output-format csv -- python3 $R/tools/prof_train_step.py --steps 8 --warmup 3 --loss-item $m > $OUT/ts_trace_$tag.log 2>&1 || { tail $OUT/ts_trace_$tag.log; exit 1; }
  f=$(find $OUT/ts_trace_$tag -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $f > $OUT/ts_timeline_$tag.txt
  grep "train step" $OUT/ts_trace_$tag.log
done
