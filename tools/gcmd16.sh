set -o pipefail
export TMPDIR=/tmp
SV_ARGS="--graph" bash tools/sv_ab.sh build build_h || exit 1
GSRAST_LIB=$(pwd)/gaussian-splatting-skysphere_amd/build_h/libgsrast.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py tests/test_gpu_bounded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt_h.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED" gpurun_out/gt_h.log | head -20; exit 1; }
tail -2 gpurun_out/gt_h.log
