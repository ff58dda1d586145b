set -o pipefail
export TMPDIR=/tmp
bash tools/sv_ab.sh build_p0 build build_b2 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_bounded.py tests/test_gpu_parity.py tests/test_render_golden.py tests/test_train_step.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" gpurun_out/gputest.log | tail -30; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
