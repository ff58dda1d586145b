"""Host-side cost of the eager rasterizer call at a small workload (C2 by default): cProfile of
N forward + backward iterations through GaussianRasterizer, sorted by own time.  The GPU work of
such a step is shorter than its Python / ctypes / allocator work, so this is where an eager C1 / C2
iteration goes."""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

WL = {"c1": (10_000, 0, 256, 256), "c2": (100_000, 3, 800, 800)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=sorted(WL))
ap.add_argument("--steps", type=int, default=300)
ap.add_argument("--capacity", type=int, default=None,
                help="bounded forwards (binning_capacity): no instance-count host wait per forward")
ap.add_argument("--no-profile", action="store_true")
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
dpix = gs_scenes.dl_dimage(H, W).to(dev)
r = GaussianRasterizer(gs_scenes.raster_settings_for(cam, deg, device=dev))


def step():
    for p in params:
        p.grad = None
    m2 = torch.zeros_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4],
               binning_capacity=a.capacity)
    img.backward(dpix)


for _ in range(20):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
print(f"{a.workload} eager{'' if a.capacity is None else f' bounded({a.capacity})'}: "
      f"{1e3 * (time.perf_counter() - t) / a.steps:.4f} ms / iteration")
if a.capacity is not None:
    import diff_gaussian_rasterization as dgr  # noqa: E402
    dgr.bounded_status()
# host time alone: each iteration after the device has drained (no overlap with kernels)
tot = 0.0
for _ in range(a.steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    step()
    tot += time.perf_counter() - t
torch.cuda.synchronize()
print(f"  launch-side time per iteration from an idle device: {1e3 * tot / a.steps:.4f} ms")
if a.no_profile:
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
