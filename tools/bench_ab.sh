#!/bin/bash
# bench.py A/B of library builds in one GPU call, alternating twice:
#   BENCH_ARGS="..." bash tools/bench_ab.sh build_a build_b ...   (dirs under gaussian-splatting-skysphere_amd/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for rep in 1 2; do
  for v in "$@"; do
    GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$v/libgsrast.so timeout -k 10 400 python bench.py --no-cpu-baseline \
      --no-train-step --no-graph --single-view-steps 0 --sustain-s 1 ${BENCH_ARGS} > $OUT/bab_$v.$rep.json 2> $OUT/bab_$v.$rep.err \
      || { echo "$v failed"; tail $OUT/bab_$v.$rep.err; exit 1; }
    python - "$OUT/bab_$v.$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
top = " ".join(f"{n}={v['total_ms_per_step']}" for n, v in sorted(k.items(), key=lambda kv: -kv[1]["total_ms_per_step"])[:7])
print(f"{sys.argv[2]:10s} value {d['value']:8.1f} sustained {d['sustained']['iters_s']:8.1f} serial {(d['serial_one_stream'] or {}).get('iters_s')} | {top}")
PY
  done
done
