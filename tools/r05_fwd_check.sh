set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_train_step.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_parity_fwdq.txt 2>&1 || { tail -30 gpurun_out/r05_parity_fwdq.txt; exit 1; }
tail -2 gpurun_out/r05_parity_fwdq.txt
SV_ARGS="" bash tools/sv_ab.sh build_base build
timeout -k 10 300 python -u tools/train_step_kernels.py > gpurun_out/r05_tsk.json 2>&1
