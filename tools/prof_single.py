"""Batch-1 step runner for rocprofv3 (bench.py's single_view shape): W warm-up + K iterations of one
view's forward + full backward into a GradBucket on one stream (C3 by default), nothing else."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

WL = {"c3": (1_000_000, 3, 1920, 1080), "c2": (100_000, 3, 800, 800), "c5": (5_000_000, 3, 1920, 1080)}

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
bucket = vp.GradBucket(params, lazy_zero=True, defer=False)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
r = GaussianRasterizer(gs_scenes.raster_settings_for(cam, deg, device=dev))
for i in range(a.warmup + a.steps):
    bucket.zero_grad()
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4])
    img.backward(dpix)
    bucket.finalize()
torch.cuda.synchronize()
print("ok")
