set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_all.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error" $OUT/gpu_all.log | head -20; tail -30 $OUT/gpu_all.log; exit 1; }
tail -2 $OUT/gpu_all.log
for rep in 1 2; do
  for bv in 0 1; do
    GSRAST_BATCH_VIEWS=$bv timeout -k 10 400 python bench.py --no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --sustain-s 1 > $OUT/bv$bv.$rep.json 2> $OUT/bv$bv.$rep.err || { echo "bench bv$bv failed"; tail $OUT/bv$bv.$rep.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$OUT/bv$bv.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
top=' '.join(f\"{n}={v['total_ms_per_step']}\" for n,v in sorted(k.items(), key=lambda kv:-kv[1]['total_ms_per_step'])[:9])
print('batch_views=$bv', d['value'], 'sust', d['sustained']['iters_s'], 'serial', (d['serial_one_stream'] or {}).get('iters_s'), '|', top)"
  done
done
for m in "" "--bounded" "--graph"; do
  timeout -k 10 200 python tools/sv_ab.py --tag build $m > $OUT/sv_mode$m.log 2>&1 || { echo "sv $m failed"; tail $OUT/sv_mode$m.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d['mode'], d['iters_s'], d['ms'], d['ksum_us'])" $OUT/sv_mode$m.log
done
timeout -k 10 400 python bench.py --workload c2 --steps 100 --no-cpu-baseline --no-train-step > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print('c2 value', d['value'], 'graph', d['graph'], 'single', d['single_view']['iters_s'])"
timeout -k 10 600 python bench.py --no-cpu-baseline --no-train-step > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -20 $OUT/bench_c3.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_c3.json').read().strip().splitlines()[-1]); print('c3 value', d['value'], 'graph', d['graph'], 'single', d['single_view']['iters_s'])"
