#!/bin/bash
# A/B library builds on the C5 bench: bash tools/ab_c5.sh build build_x ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for b in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$b/libgsrast.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload c5 > $OUT/ab5_$b.log 2>&1 || { echo "bench $b failed"; tail $OUT/ab5_$b.log; exit 1; }
  python - $b <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab5_{sys.argv[1]}.log") if l.startswith("{")][0])
print(f"c5 {sys.argv[1]:10s} value {d['value']:8.2f} ms {d['ms_per_step']:.4f}", {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done
