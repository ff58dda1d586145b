#!/bin/bash
# bench.py variants in one GPU call: bash tools/variants.sh "<args 1>" "<args 2>" ...  (value + ms per step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps ${V_STEPS:-50} --warmup 5 --no-cpu-baseline --no-train-step $a > $OUT/var_$i.log 2>&1 || { echo "variant '$a' failed"; tail $OUT/var_$i.log; exit 1; }
  python - "$OUT/var_$i.log" "$a" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(f"{sys.argv[2]:45s} value {d['value']:8.1f} ms/step {d['ms_per_step']:.4f} sustained {d['sustained']['iters_s']}")
PY
done
