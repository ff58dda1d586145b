set -o pipefail
export TMPDIR=/tmp
SV_ARGS="--graph" bash tools/sv_ab.sh build build_d256 build_d128 || exit 1
