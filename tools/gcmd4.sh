set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiview.py tests/test_gpu_bounded.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_mv.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_mv.log; exit 1; }
tail -1 $OUT/gpu_mv.log
for wl in c5; do
for rep in 1 2; do
  for bv in 0 1; do
    GSRAST_BATCH_VIEWS=$bv timeout -k 10 400 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --sustain-s 1 > $OUT/bv_${wl}_$bv.$rep.json 2> $OUT/bv_${wl}_$bv.$rep.err || { echo "bench $wl bv$bv failed"; tail $OUT/bv_${wl}_$bv.$rep.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$OUT/bv_${wl}_$bv.$rep.json').read().strip().splitlines()[-1]); k=d['kernels']
top=' '.join(f\"{n}={v['total_ms_per_step']}\" for n,v in sorted(k.items(), key=lambda kv:-kv[1]['total_ms_per_step'])[:8])
print('$wl batch_views=$bv', d['value'], 'sust', d['sustained']['iters_s'], 'serial', (d['serial_one_stream'] or {}).get('iters_s'), '|', top)"
  done
done
done
bash tools/sv_ab.sh build_sr0 build_s1 build_s2 build_s3 build_sr || exit 1
GSRAST_LIB=$PWD/gaussian-splatting-skysphere_amd/build_sr/libgsrast.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiview.py tests/test_gpu_bounded.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_sr.log 2>&1 || { echo "sr tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_sr.log | head; tail -30 gpurun_out/gpu_sr.log; exit 1; }
tail -1 gpurun_out/gpu_sr.log
