#!/bin/bash
# Batch-1 A/B of library builds in one GPU call, alternating twice:
#   bash tools/sv_ab.sh build_a build_b ...   (directories under gaussian-splatting-skysphere_amd/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for rep in 1 2; do
  for v in "$@"; do
    GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$v/libgsrast.so timeout -k 10 200 python tools/sv_ab.py --tag $v ${SV_ARGS} > $OUT/sv_$v.$rep.log 2>&1 || { echo "$v failed"; tail $OUT/sv_$v.$rep.log; exit 1; }
    python - "$OUT/sv_$v.$rep.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
k = d["kernels"]
top = " ".join(f"{n}={v}" for n, v in list(k.items())[:6])
print(f"{d['tag']:14s} {d['mode']:9s} {d['iters_s']:7.1f} it/s {d['ms']:.4f} ms ksum {d['ksum_us']} | {top}")
PY
  done
done
