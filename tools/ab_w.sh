#!/bin/bash
# A/B library builds on one workload: WL=c2 bash tools/ab_w.sh build build_x ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
WL=${WL:-c3}
for b in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$b/libgsrast.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --workload $WL > $OUT/abw_${WL}_$b.log 2>&1 || { echo "bench $b failed"; tail $OUT/abw_${WL}_$b.log; exit 1; }
  python - $b $WL <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/abw_{sys.argv[2]}_{sys.argv[1]}.log") if l.startswith("{")][0])
print(f"{sys.argv[2]} {sys.argv[1]:10s} value {d['value']:8.2f} ms {d['ms_per_step']:.4f}", {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done
