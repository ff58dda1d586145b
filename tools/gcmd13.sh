set -o pipefail
export TMPDIR=/tmp
SV_ARGS="--graph" bash tools/sv_ab.sh build build_w2 build_w8 || exit 1
