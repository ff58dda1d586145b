set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bounded.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_bounded.log 2>&1 || { echo "bounded tests failed"; tail -40 $OUT/gpu_bounded.log; exit 1; }
tail -3 $OUT/gpu_bounded.log
for m in "" "--bounded" "--graph"; do
  timeout -k 10 200 python tools/sv_ab.py --tag build $m > $OUT/sv_mode$m.log 2>&1 || { echo "sv $m failed"; tail $OUT/sv_mode$m.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d['mode'], d['iters_s'], d['ms'], d['ksum_us'])" $OUT/sv_mode$m.log
done
for m in "" "--graph"; do
  timeout -k 10 200 python tools/sv_ab.py --workload c2 --tag c2 $m > $OUT/sv_c2$m.log 2>&1 || { echo "sv c2 $m failed"; tail $OUT/sv_c2$m.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print('c2', d['mode'], d['iters_s'], d['ms'], d['ksum_us'])" $OUT/sv_c2$m.log
done
timeout -k 10 400 python bench.py --workload c2 --steps 100 --no-cpu-baseline --no-train-step > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2 value', d['value'], 'graph', d['graph'], 'single', d['single_view']['iters_s'])"
timeout -k 10 500 python bench.py --no-cpu-baseline --no-train-step > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -20 $OUT/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c3.json')); print('c3 value', d['value'], 'graph', d['graph'], 'single', d['single_view']['iters_s'])"
