cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiview.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mv.log 2>&1; rc=$?
tail -2 gpurun_out/mv.log; grep -E "^E  .*Error|FAILED|^E  " gpurun_out/mv.log | head -8
[ $rc -eq 0 ] || exit $rc
for a in "--no-defer" ""; do
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $a > gpurun_out/b.json 2>gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$a', d['value'], d['ms_per_step'], d['sustained']['iters_s'], d['serial_one_stream'], {k:(v['avg_us'],v['launches_per_step']) for k,v in d['kernels'].items() if 'bwd' in k or 'gauss' in k or 'mean2d' in k or 'sum' in k}, d['step_roofline']['frac'])"
done
