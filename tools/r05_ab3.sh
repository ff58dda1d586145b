# round 5: parity subset on the current build, then batch-1 A/B of three builds
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ext.py tests/test_train_step.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_parity_sub.txt 2>&1 || { tail -30 gpurun_out/r05_parity_sub.txt; exit 1; }
tail -1 gpurun_out/r05_parity_sub.txt
SV_ARGS="" bash tools/sv_ab.sh build_base build build_c
