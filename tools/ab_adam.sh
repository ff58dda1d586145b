#!/bin/bash
# Kernel-time A/B of library variants on the C3 train step: bash tools/ab_adam.sh build build_x ...
# (each a build directory under gaussian-splatting-skysphere_amd/, made with make BUILD=... EXTRA=...)
set -e
R=$GRAFT_REPO_ROOT; cd /tmp; export TMPDIR=/tmp
for v in "$@"; do
  GSRAST_LIB=$R/gaussian-splatting-skysphere_amd/$v/libgsrast.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$v -o ts -- python $R/tools/prof_train_step.py --steps 30 --warmup 5 > $R/gpurun_out/ab_$v.log 2>&1
  python - $R/gpurun_out/ab_$v/ts_kernel_stats.csv $v <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = 35
tot = sum(float(r['TotalDurationNs']) for r in rows) / n / 1e3
pick = {r['Name'].split('(')[0].split('::')[-1].split('<')[0]: float(r['TotalDurationNs']) / n / 1e3 for r in rows}
keys = ['k_adam', 'k_activate_fwd', 'k_activate_bwd', 'k_preprocess', 'k_preprocess_bwd_reg', 'k_render_fwd_q', 'k_render_bwd']
print(f"{sys.argv[2]:14s} total {tot:7.1f} us/iter  " + "  ".join(f"{k[2:]} {pick.get(k, 0):.1f}" for k in keys))
PY
done
