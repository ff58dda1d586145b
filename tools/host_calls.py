"""Host time of the eager rasterizer calls at a small workload (C2 by default), call by call:
the extension's forward (two-call path vs gs_forward_counted) and backward, each timed from an
idle device (torch.cuda.synchronize() before every call) and in a back-to-back loop."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

WL = {"c1": (10_000, 0, 256, 256), "c2": (100_000, 3, 800, 800), "c3": (1_000_000, 3, 1920, 1080)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=sorted(WL))
ap.add_argument("--steps", type=int, default=300)
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
s = gs_scenes.raster_settings_for(cam, deg, device=dev)
e = torch.empty(0, device=dev)
args = (s.bg, sc.means3D, e, sc.opacities, sc.scales, sc.rotations, 1.0, e, s.viewmatrix, s.projmatrix, s.tanfovx,
        s.tanfovy, H, W, sc.shs, deg, s.campos, False, False)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
X = _C._EXT
assert X is not None


def fwd(counted):
    if not counted:
        X.set_count_estimate(0, P, W, H, 0)
    return X.forward(*args[:-1], args[-1], None)


def bwd(out):
    nr, color, radii, geom, binning, img = out
    return X.backward(s.bg, sc.means3D, radii, e, sc.scales, sc.rotations, 1.0, e, s.viewmatrix, s.projmatrix,
                      s.tanfovx, s.tanfovy, dpix, sc.shs, deg, s.campos, geom, nr, binning, img, False, None)


def timed(fn, idle, n):
    tot = 0.0
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        if idle:
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            tot += time.perf_counter() - t
        else:
            fn()
    torch.cuda.synchronize()
    return 1e6 * (tot if idle else time.perf_counter() - t0) / n


for counted in (False, True):
    tag = "counted " if counted else "two-call"
    print(f"{tag} forward  from idle: {timed(lambda: fwd(counted), True, a.steps):8.1f} us   "
          f"back-to-back: {timed(lambda: fwd(counted), False, a.steps):8.1f} us")
    out = fwd(counted)
    torch.cuda.synchronize()
    print(f"{tag} backward from idle: {timed(lambda: bwd(out), True, a.steps):8.1f} us   "
          f"back-to-back: {timed(lambda: bwd(out), False, a.steps):8.1f} us")
    print(f"{tag} fwd+bwd  from idle: {timed(lambda: bwd(fwd(counted)), True, a.steps):8.1f} us   "
          f"back-to-back: {timed(lambda: bwd(fwd(counted)), False, a.steps):8.1f} us")
print("estimate", X.count_estimate(0, P, W, H), "num_rendered", out[0])
