# round 5: full GPU suite (kernel coverage last), batch-1 A/B of the base build against the
# current one, train-step kernel profile, default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_gpu_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r05_gpu_tests.txt
if [ $rc -ne 0 ]; then
  # only the kernel-coverage listing failed (it runs last): report it and go on to the measurements
  if grep -q "^1 failed" gpurun_out/r05_gpu_tests.txt && grep -q "FAILED tests/test_zz_kernel_coverage" gpurun_out/r05_gpu_tests.txt; then
    sed -n '/never launched/,$p' gpurun_out/kernel_coverage.txt
  else
    grep -E "FAILED|Error|assert" gpurun_out/r05_gpu_tests.txt | head -20; exit 1
  fi
fi
SV_ARGS="" bash tools/sv_ab.sh ${BASE:-build} build || exit 1
timeout -k 10 200 python -u tools/train_step_kernels.py > gpurun_out/r05_tsk.json 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err
