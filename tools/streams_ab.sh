# Alternating bench runs of the C3 4-view step with 2 / 3 / 4 view streams (bench.py --streams).
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for s in 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step --no-graph --single-view-steps 0 --steps 100 --streams $s > gpurun_out/st_$s.$rep.json 2> gpurun_out/st_$s.$rep.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/st_$s.$rep.json'))
print('streams $s value %8.1f sustained %8.1f' % (d['value'], d['sustained']['iters_s']))"
done; done
