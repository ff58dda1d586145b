#!/bin/bash
# PMC passes over the batch-1 loop (tools/prof_single.py), one rocprofv3 run per counter group
# (--kernel-trace only beside --pmc), restricted to the kernels matching $KRE (default render).
# Output: gpurun_out/pmcs_<name>/...; summary via tools/pmc_summary.py gpurun_out pmcs_.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $OUT
cd /tmp
KRE=${KRE:-render}
run() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex "$KRE" --pmc "$@" -d $OUT/pmcs_$name -o run \
    --output-format csv -- python3 $R/tools/prof_single.py --steps 4 --warmup 1 > $OUT/pmcs_$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH || exit 1
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
echo pmc done
