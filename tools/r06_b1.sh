cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
GS_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --workload c2 --steps 20 --warmup 3 --no-graph --single-view-steps 0 --sustain-s 0 --regions 1 > gpurun_out/r06_b1_c2_gloo2.json 2> gpurun_out/r06_b1_c2_gloo2.err && \
timeout -k 10 400 python bench.py > gpurun_out/r06_b1_c3.json 2> gpurun_out/r06_b1_c3.err
