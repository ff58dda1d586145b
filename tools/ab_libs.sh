#!/bin/bash
# bench.py A/B of library builds in one GPU call: bash tools/ab_libs.sh "<bench args>" build_a build_b ...
# (each a build directory under gaussian-splatting-skysphere_amd/, made with make BUILD=... EXTRA=...)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
args=$1; shift
for v in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$v/libgsrast.so timeout -k 10 300 python bench.py --steps ${V_STEPS:-50} --warmup 5 --no-cpu-baseline --no-train-step $args > $OUT/ab_$v.log 2>&1 || { echo "$v failed"; tail $OUT/ab_$v.log; exit 1; }
  python - "$OUT/ab_$v.log" "$v $args" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
k = d["kernels"]
print(f"{sys.argv[2]:28s} value {d['value']:8.1f} ms/step {d['ms_per_step']:.4f} scatter {k['radix_scatter']['avg_us']:.2f} hist {k['radix_hist']['avg_us']:.2f}")
PY
done
