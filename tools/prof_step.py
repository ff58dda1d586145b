"""Minimal step runner for rocprofv3 PMC passes: W warmup + K rasterizer fwd+bwd steps of a
bench workload (default C3), nothing else on the GPU."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

WL = {"c3": (1_000_000, 3, 1920, 1080), "c2": (100_000, 3, 800, 800), "c5": (5_000_000, 3, 1920, 1080)}

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--warmup", type=int, default=1)
ap.add_argument("--forward-only", action="store_true")
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
s = gs_scenes.raster_settings_for(cam, deg, device=dev)
params = [t.clone().requires_grad_(not a.forward_only) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
m2 = torch.zeros_like(params[0], requires_grad=not a.forward_only)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
r = GaussianRasterizer(s)
for i in range(a.warmup + a.steps):
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4])
    if not a.forward_only:
        img.backward(dpix)
        for p in params + [m2]:
            p.grad = None
torch.cuda.synchronize()
print("ok")
