set -o pipefail
export TMPDIR=/tmp
GSRAST_SLABS=2 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest_slabs2.log 2>&1
rc=$?
tail -30 gpurun_out/gputest_slabs2.log
exit 0
