set -o pipefail
cd $GRAFT_REPO_ROOT
export GSRAST_LIB=$PWD/gaussian-splatting-skysphere_amd/build_timing/libgsrast.so
timeout -k 10 240 python -u tools/bwd_timing.py --workload c3 --reps 3 --out gpurun_out/bwd_timing_c3.json > gpurun_out/bwd_timing_c3.log 2>&1 &&
timeout -k 10 240 python -u tools/bwd_timing.py --workload c5 --reps 2 --out gpurun_out/bwd_timing_c5.json > gpurun_out/bwd_timing_c5.log 2>&1
