"""Batch-1 A/B timer: the single-view loop of bench.py (one view's forward + full backward into a
GradBucket, one stream) with the library named by $GSRAST_LIB; prints iters/s and per-kernel HIP-event
times.  tools/sv_ab.sh runs it for several builds, alternating."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native, bounded_status, last_num_rendered  # noqa: E402

WL = {"c3": (1_000_000, 3, 1920, 1080), "c2": (100_000, 3, 800, 800), "c5": (5_000_000, 3, 1920, 1080)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--tag", default="")
ap.add_argument("--bounded", action="store_true", help="bounded forwards (capacity = measured count x 1.1 + 4096)")
ap.add_argument("--graph", action="store_true", help="bounded, and the step captured into a HIP graph")
ap.add_argument("--no-prof", action="store_true", help="skip the per-kernel event pass (for an external profiler)")
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
bucket = vp.GradBucket(params, lazy_zero=True, defer=False)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
r = GaussianRasterizer(gs_scenes.raster_settings_for(cam, deg, device=dev))


cap = None


def eager_step():
    bucket.zero_grad()
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4],
               binning_capacity=cap)
    img.backward(dpix)
    bucket.finalize()


step = eager_step
for _ in range(10):
    step()
torch.cuda.synchronize()
if a.bounded or a.graph:
    cap = int(last_num_rendered() * 1.1) + 4096
    for _ in range(3):
        step()
    torch.cuda.synchronize()
if a.graph:
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        eager_step()
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(graph):
        eager_step()
    step = graph.replay
    for _ in range(3):
        step()
    torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / a.steps
if cap is not None:
    bounded_status()  # raises if a view outgrew its capacity
    step = eager_step  # (per-kernel events: eager launches)
if a.no_prof:
    print(json.dumps({"tag": a.tag, "iters_s": round(1 / dt, 1), "ms": round(1e3 * dt, 4)}))
    sys.exit(0)
lib = _native.load()
lib.gs_profile_reset()
lib.gs_profile_enable(1)
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
lib.gs_profile_enable(0)
prof = _native.profile_stats()
k = {n: round(1e3 * ms / a.steps, 2) for n, (ms, c) in sorted(prof.items(), key=lambda kv: -kv[1][0])}
print(json.dumps({"tag": a.tag, "lib": os.environ.get("GSRAST_LIB", "default"), "iters_s": round(1 / dt, 1),
                  "ms": round(1e3 * dt, 4), "ksum_us": round(sum(k.values()), 1), "mode": "graph" if a.graph else
                  "bounded" if a.bounded else "read-back", "kernels": k}))
