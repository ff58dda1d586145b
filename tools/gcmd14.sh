set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.log; exit 1; }
timeout -k 10 400 python bench.py --workload c4 --c4-views-per-rank 4 --steps 20 --warmup 3 --no-cpu-baseline --no-train-step > $OUT/bench_c4w.log 2>&1 || { echo "bench c4 weak failed"; tail -20 $OUT/bench_c4w.log; exit 1; }
timeout -k 10 300 python bench.py --workload c1 --steps 20 --warmup 3 > $OUT/bench_c1.log 2>&1 || { echo "bench c1 failed"; tail -20 $OUT/bench_c1.log; exit 1; }
for f in bench_c4 bench_c4w bench_c1; do python -c "
import json; d=json.loads([l for l in open('$OUT/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['unit'], d['ms_per_step'], d['scaling'], d['config'].get('views_per_step'), (d.get('graph') or {}).get('step'), (d.get('cpu_baseline') or {}).get('value'))"; done
