#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
SV_ARGS="--steps 30" timeout -k 10 400 bash tools/sv_ab.sh build_e2 build_e4 build_d build > $OUT/r05_sv_ab4.txt 2>&1 || { cat $OUT/r05_sv_ab4.txt; exit 1; }
cat $OUT/r05_sv_ab4.txt
GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/build_timing_inf/libgsrast.so timeout -k 10 200 python -u tools/fwd_timing.py --workload c3 --reps 2 --out $OUT/r05_fwd_timing_inf.json > $OUT/r05_fwd_timing_inf.log 2>&1 || { tail $OUT/r05_fwd_timing_inf.log; exit 1; }
grep -v amdgpu.ids $OUT/r05_fwd_timing_inf.log
