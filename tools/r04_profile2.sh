#!/bin/bash
# Round-4 profile set, part 2 (one GPU call): the PMC passes over bench.py's step (tools/pmc_passes.sh,
# for profiles/pmc_traffic.json / pmc_valu.json), and kernel stats (no counters) of the batch-1
# rasterizer loop and of the train step, for render_bwd in the two contexts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04p2
export TMPDIR=/tmp
mkdir -p $O
bash $R/tools/pmc_passes.sh || exit 1
cd /tmp
for s in prof_single prof_train_step; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$s -o run -- \
    python3 $R/tools/$s.py --steps 30 --warmup 3 > $O/ks_$s.log 2>&1 || { echo "$s failed"; tail $O/ks_$s.log; exit 1; }
  rm -f $O/ks_$s/run_kernel_trace.csv
  echo "$s done"
done
