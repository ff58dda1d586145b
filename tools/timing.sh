#!/bin/bash
# Critical-path timing of both render kernels from the -DGS_TIMING build (TAG names the outputs):
#   make -C gaussian-splatting-skysphere_amd BUILD=build_timing EXTRA=-DGS_TIMING; TAG=x bash tools/timing.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/build_timing/libgsrast.so
timeout -k 10 200 python -u tools/bwd_timing.py --workload c3 --reps 2 --out $OUT/bwd_timing_${TAG}.json > $OUT/bwd_timing_${TAG}.log 2>&1 || { tail $OUT/bwd_timing_${TAG}.log; exit 1; }
grep -v amdgpu.ids $OUT/bwd_timing_${TAG}.log
timeout -k 10 200 python -u tools/fwd_timing.py --workload c3 --reps 2 --out $OUT/fwd_timing_${TAG}.json > $OUT/fwd_timing_${TAG}.log 2>&1 || { tail $OUT/fwd_timing_${TAG}.log; exit 1; }
grep -v amdgpu.ids $OUT/fwd_timing_${TAG}.log
