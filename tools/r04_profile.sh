#!/bin/bash
# Round-4 profile set (one GPU call): the default C3 bench line; rocprofv3 kernel stats of exactly
# the bench's one-stream kernel-duration pass (bench.py --profile-pass-only: roofline.frac is
# recomputable from it); PMC passes on render_bwd in the rasterizer loop (prof_single.py) and in the
# train step (prof_train_step.py).  Outputs under gpurun_out/r04p/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04p
export TMPDIR=/tmp
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail $O/bench_c3.err; exit 1; }
echo "bench done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pass -o run -- \
  python3 $R/bench.py --profile-pass-only --steps 50 --warmup 2 > $O/pass.json 2> $O/pass.err || { echo "pass failed"; tail $O/pass.err; exit 1; }
rm -f $O/pass/run_kernel_trace.csv
echo "profile pass done"
pmc() {
  name=$1; script=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex render_bwd --pmc "$@" -d $O/pmc_$name -o run \
    --output-format csv -- python3 $R/tools/$script --steps 4 --warmup 2 > $O/pmc_$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
pmc sq_single prof_single.py $SQ || exit 1
pmc sq_train prof_train_step.py $SQ || exit 1
pmc fetch_single prof_single.py FETCH_SIZE || exit 1
pmc fetch_train prof_train_step.py FETCH_SIZE || exit 1
echo "pmc done"
