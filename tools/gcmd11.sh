set -o pipefail
export TMPDIR=/tmp
bash tools/sv_ab.sh build build_p build_p4 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiview.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/mv.log 2>&1 || { echo "multiview tests failed"; tail -30 gpurun_out/mv.log; exit 1; }
tail -2 gpurun_out/mv.log
