"""Host-side cost of bench.py's multi-view step (fused front, K views on 2 streams, backwards into
a deferred GradBucket) at a small workload: cProfile of N steps with the autograd engine in the
calling thread (torch.autograd.set_multithreading_enabled(False)) so the backward's Python shows."""
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
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, prepare_views  # noqa: E402

WL = {"c1": (10_000, 0, 256, 256), "c2": (100_000, 3, 800, 800)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=sorted(WL))
ap.add_argument("--steps", type=int, default=300)
ap.add_argument("--views", type=int, default=4)
ap.add_argument("--sort", default="tottime")
ap.add_argument("--capacity", type=int, default=None, help="bounded views (binning_capacity): no count readback")
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--lines", type=int, default=40)
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
cams = gs_scenes.jittered_cameras(a.views, W, H, seed=7)
cams[0] = cam
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
dpix = gs_scenes.dl_dimage(H, W, seed=1).to(dev)
rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, deg, device=dev)) for c in cams]
bucket = vp.GradBucket(params, lazy_zero=True, defer=True, chunks=1)
streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]


def view_fn(r, pre):
    def run():
        m2 = torch.empty_like(params[0], requires_grad=True)
        img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                   rotations=params[4], prepared=pre)
        img.backward(dpix)
    return run


def step():
    bucket.zero_grad()
    pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4],
                        streams=[streams[k % len(streams)] for k in range(len(rasts))], binning_capacity=a.capacity)
    vp.run_views([view_fn(r, p) for r, p in zip(rasts, pre)], streams)
    bucket.finalize()


for _ in range(20):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / a.steps
print(f"{a.workload} {a.views}-view step: {1e3 * dt:.4f} ms ({a.views / dt:.1f} views/s)")
tot = 0.0
for _ in range(a.steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    step()
    tot += time.perf_counter() - t
torch.cuda.synchronize()
print(f"  launch-side time per step from an idle device: {1e3 * tot / a.steps:.4f} ms")
torch.autograd.set_multithreading_enabled(False)
pr = cProfile.Profile()
pr.enable()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats(a.sort).print_stats(a.lines)
