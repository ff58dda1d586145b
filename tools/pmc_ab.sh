#!/bin/bash
# PMC passes of the render kernels for several library builds (batch-1 loop, tools/prof_single.py).
#   bash tools/pmc_ab.sh build build_r4 ...      -> gpurun_out/pmcab_<build>_<pass>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
KRE=${KRE:-render}
for b in "$@"; do
  export GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$b/libgsrast.so
  run() {
    name=$1; shift
    timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex "$KRE" --pmc "$@" -d $OUT/pmcab_${b}_$name -o run \
      --output-format csv -- python3 $R/tools/prof_single.py --steps 4 --warmup 1 > $OUT/pmcab_${b}_$name.log 2>&1
    rc=$?; echo "$b pass $name rc=$rc"; return $rc
  }
  run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
  run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH || exit 1
  run fetch FETCH_SIZE || exit 1
  run write WRITE_SIZE || exit 1
  run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
done
echo pmc done
