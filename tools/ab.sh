#!/bin/bash
# A/B library builds on the bench (same process settings, sequential runs): bash tools/ab.sh build build_x ...
# Each build dir is gaussian-splatting-skysphere_amd/<dir> (make BUILD=<dir> EXTRA=-D...).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for b in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$b/libgsrast.so timeout -k 10 300 python bench.py --steps ${AB_STEPS:-100} --warmup 10 --no-cpu-baseline > $OUT/ab_$b.log 2>&1 || { echo "bench $b failed"; tail $OUT/ab_$b.log; exit 1; }
  python - $b <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][0])
print(f"{sys.argv[1]:12s} value {d['value']:8.2f} ms {d['ms_per_step']:.4f}", {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done
echo ab done
