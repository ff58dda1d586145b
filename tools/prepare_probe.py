"""Host time of prepare_views at C2 (4 views) from an idle device: the counted call (host waits for
the views' instance counts) against the bounded call (no readback), and the ext call alone.
    python tools/prepare_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, prepare_views, last_num_rendered  # noqa: E402

P, deg, W, H = 100_000, 3, 800, 800
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
cams = gs_scenes.jittered_cameras(4, W, H, seed=7)
cams[0] = cam
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, deg, device=dev)) for c in cams]
streams = [torch.cuda.Stream(dev) for _ in range(2)]
sts = [streams[k % 2] for k in range(4)]
pc = time.perf_counter


def run(n, **kw):
    tot = 0.0
    for _ in range(n):
        torch.cuda.synchronize()
        t = pc()
        prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4],
                      streams=sts, **kw)
        tot += pc() - t
    torch.cuda.synchronize()
    return 1e6 * tot / n


pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4], streams=sts)
cap = int(pre[0].triple[0] * 1.2)
for rep in range(3):
    a = run(200)
    b = run(200, binning_capacity=cap)
    print(f"prepare_views from idle: counted {a:7.1f} us   bounded (no readback) {b:7.1f} us")
# GPU time of the front (preprocess + orderings + binning), events on the current stream
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(50):
    prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4])
e1.record()
torch.cuda.synchronize()
print(f"front GPU+host per call on one stream, back to back: {1e3 * e0.elapsed_time(e1) / 50:.1f} us")
