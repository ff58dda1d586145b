cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?
tail -2 gpurun_out/gputest.log; grep -E "^E  .*Error|FAILED" gpurun_out/gputest.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'], d['ms_per_step'], d['sustained'], d['serial_one_stream'], d['cpu_baseline']['value'])"
