set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
grep -h "OK\|FAIL" /tmp/pytest-of-*/pytest-*/*/vp_*.txt 2>/dev/null | head -5
bash tools/sv_ab.sh build build_a1 build_a2 build_a3
GS_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --single-view-steps 0 > gpurun_out/bench_gloo2.log 2>&1 || { echo "gloo2 bench failed"; tail -20 gpurun_out/bench_gloo2.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_gloo2.log") if l.startswith("{")][0])
print("gloo2", d["n_gpus"], d["value"], d["config"]["parallelism"])
PY
