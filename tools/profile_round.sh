# Round profile set (each GPU step has its own limit; stops at the first failure):
# C3 bench line, rocprofv3 stats of the bench's one-stream event pass (roofline.frac), PMC passes
# (traffic + SQ counters of every kernel), batch-1 rocprof kernel stats, C2 and C5 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/profile_${TAG:-round}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -20 $OUT/bench_c3.err; exit 1; }
echo "bench c3 ok"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_pass -o run --output-format csv -- python3 $R/bench.py --profile-pass-only --steps 100 --warmup 10 > $OUT/profile_pass.json 2> $OUT/profile_pass.err || { echo "rocprof pass failed"; tail -20 $OUT/profile_pass.err; exit 1; }
echo "rocprof pass ok"
cd $R
GRAFT_REPO_ROOT=$R bash tools/pmc_passes.sh > $OUT/pmc_passes.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc_passes.log; exit 1; }
python3 tools/pmc_traffic.py $R/gpurun_out c3 $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1 || { echo "pmc_traffic failed"; exit 1; }
python3 tools/pmc_summary.py $R/gpurun_out > $OUT/pmc_summary.txt 2>&1
echo "pmc ok"
STEPS=20 bash tools/prof_single.sh > $OUT/prof_single.txt 2>&1 || { echo "prof single failed"; tail $OUT/prof_single.txt; exit 1; }
echo "prof single ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --workload c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.err; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench c5 failed"; tail -20 $OUT/bench_c5.err; exit 1; }
echo done
