set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; export TMPDIR=/tmp; mkdir -p $OUT; cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  name=$( [ $ctr = FETCH_SIZE ] && echo fetch || echo write )
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/pmc_$name -o run --output-format csv -- python3 $R/tools/prof_step.py --workload c3 --steps 2 --warmup 1 > $OUT/pmc_$name.log 2>&1 || exit 1
done
python3 $R/tools/pmc_traffic.py $OUT c3 $OUT/pmc_traffic_rec.json
