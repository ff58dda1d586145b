set -o pipefail
export TMPDIR=/tmp
bash tools/sv_ab.sh build build_g || exit 1
SV_ARGS="--graph" bash tools/sv_ab.sh build build_g || exit 1
GSRAST_LIB=$(pwd)/gaussian-splatting-skysphere_amd/build_g/libgsrast.so bash tools/gpu_tests.sh -x -q || exit 1
