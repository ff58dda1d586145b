set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_slabs.py tests/test_gpu_bounded.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_slabs.log 2>&1 || { echo "slab tests failed"; grep -E "FAIL|Error|assert" $OUT/gpu_slabs.log | head -20; tail -40 $OUT/gpu_slabs.log; exit 1; }
grep -E "passed|slabs\]" $OUT/gpu_slabs.log | tail -3
bash tools/sv_ab.sh build_sr0 build_s1 build_s2 build || exit 1
for rep in 1 2; do
  for sl in 0 1; do
    GSRAST_SLABS=$sl timeout -k 10 400 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --sustain-s 1 > $OUT/sl_c5_$sl.$rep.json 2> $OUT/sl_c5_$sl.$rep.err || { echo "bench c5 slabs=$sl failed"; tail $OUT/sl_c5_$sl.$rep.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/sl_c5_$sl.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
top=' '.join(f\"{n}={v['total_ms_per_step']}\" for n,v in sorted(k.items(), key=lambda kv:-kv[1]['total_ms_per_step'])[:10])
print('c5 slabs=$sl', d['value'], 'sust', d['sustained']['iters_s'], 'serial', (d['serial_one_stream'] or {}).get('iters_s'), '|', top)"
  done
done
