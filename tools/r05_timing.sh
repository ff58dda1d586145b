#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/build_timing/libgsrast.so
timeout -k 10 200 python -u tools/bwd_timing.py --workload c3 --reps 2 --out $OUT/r05_bwd_timing_${TAG}.json > $OUT/r05_bwd_timing_${TAG}.log 2>&1 || { tail $OUT/r05_bwd_timing_${TAG}.log; exit 1; }
grep -v amdgpu.ids $OUT/r05_bwd_timing_${TAG}.log
timeout -k 10 200 python -u tools/fwd_timing.py --workload c3 --reps 2 --out $OUT/r05_fwd_timing_${TAG}.json > $OUT/r05_fwd_timing_${TAG}.log 2>&1 || { tail $OUT/r05_fwd_timing_${TAG}.log; exit 1; }
grep -v amdgpu.ids $OUT/r05_fwd_timing_${TAG}.log
