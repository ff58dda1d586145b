#!/bin/bash
# Round-4 backward check in one GPU call: the GPU parity suite on the default build (stops at the
# first failure), then a batch-1 A/B of the default build against the builds named as arguments
# (directories under gaussian-splatting-skysphere_amd/, e.g. build_old = make EXTRA=-DGS_BWD_TW=0).
#   bash tools/r04_bwd.sh [build_x ...]      env: TESTS (pytest selection, default: the whole -m gpu suite)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/r04_tests.log 2>&1
rc=$?
tail -4 $OUT/r04_tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -m5 -E "FAILED|Error" $OUT/r04_tests.log; exit $rc; }
[ $# -gt 0 ] && bash tools/sv_ab.sh build "$@"
