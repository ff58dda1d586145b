set -o pipefail
cd $GRAFT_REPO_ROOT
for v in build build_hwexp build; do
  GSRAST_LIB=$PWD/gaussian-splatting-skysphere_amd/$v/libgsrast.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
  python - $v <<'PY'
import json,sys
d=json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][0])
print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items() if k.startswith("render")})
PY
done
