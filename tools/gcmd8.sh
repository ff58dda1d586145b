set -o pipefail
export TMPDIR=/tmp
bash tools/sv_ab.sh build_base build || exit 1
bash tools/gpu_tests.sh -x -q || exit 1
