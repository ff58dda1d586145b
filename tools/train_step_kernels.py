"""Per-kernel device time of one train.py iteration (gs_train_step.train_step, loss.item() per
iteration) with and without the fused-Adam backward, on bench.py's C3 scene: the library's own
event profile (gs_profile_*) over N iterations, printed as JSON (us per iteration per kernel) with
the wall-clock iteration rate of the same loop."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_train_step as ts  # noqa: E402
from diff_gaussian_rasterization import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(a.W, a.H)
sc = gs_scenes.random_gaussians(a.P, 3, cam=cam, seed=0)
settings = gs_scenes.raster_settings_for(cam, 3, device=dev)
gt = torch.rand((3, a.H, a.W), generator=torch.Generator().manual_seed(2)).to(dev)
lib = _native.load()
out = {}
for fuse in (False, True):
    m = ts.TrainModel(sc, dev, fused=True)
    for _ in range(3):
        ts.train_step(m, settings, gt, loss_item=True, fuse_adam=fuse)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        ts.train_step(m, settings, gt, loss_item=True, fuse_adam=fuse)
    dt = (time.perf_counter() - t) / a.iters
    lib.gs_profile_reset()
    lib.gs_profile_enable(1)
    for _ in range(a.iters):
        ts.train_step(m, settings, gt, loss_item=True, fuse_adam=fuse)
    torch.cuda.synchronize()
    lib.gs_profile_enable(0)
    st = _native.profile_stats()
    ks = {k: round(1e3 * v[0] / a.iters, 2) for k, v in sorted(st.items(), key=lambda kv: -kv[1][0])}
    out["fused_adam" if fuse else "unfused"] = {"iters_s": round(1 / dt, 1), "kernel_us": ks,
                                                "kernel_us_sum": round(sum(ks.values()), 1)}
    del m
print(json.dumps(out, indent=1))
