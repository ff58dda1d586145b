#!/bin/bash
# Alternating A/B of host-side (Python / ext) changes: this tree against a copy of the package under
# ab_old/ (git archive of the base commit, its ext built there), tools/host_phases.py three times each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/build/libgsrast.so
for rep in 1 2 3; do
  timeout -k 10 120 python tools/host_phases.py ${HP_ARGS} > $OUT/hp_new.$rep.log 2>&1 || { tail $OUT/hp_new.$rep.log; exit 1; }
  GS_PKG=$R/ab_old/gaussian-splatting-skysphere_amd timeout -k 10 120 python tools/host_phases.py ${HP_ARGS} > $OUT/hp_old.$rep.log 2>&1 || { tail $OUT/hp_old.$rep.log; exit 1; }
  for v in new old; do echo "== $v $rep"; grep -v amdgpu.ids $OUT/hp_$v.$rep.log | tail -n +2; done
done
