set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
run() {  # $1 tag, env in the caller
  timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --sustain-s 1 > $OUT/sw_$1.json 2> $OUT/sw_$1.err || { echo "bench $1 failed"; tail $OUT/sw_$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/sw_$1.json').read().strip().splitlines()[-1]); k=d['kernels']
top=' '.join(f\"{n}={v['total_ms_per_step']}\" for n,v in sorted(k.items(), key=lambda kv:-kv[1]['total_ms_per_step'])[:16])
print('$1', d['value'], '|', top)"
}
GSRAST_SLABS=0 run off || exit 1
for n in 8 12 16 24 32 40; do GSRAST_SLABS=1 GSRAST_SLAB_NEAR64=$n run n$n || exit 1; done
GSRAST_SLABS=0 run off2 || exit 1
