"""Instrumentation: distribution of contributing lanes per walked backward entry at C3.
Needs a library built with -DGS_BWD_STATS (make BUILD=build_stats EXTRA=-DGS_BWD_STATS) and
GSRAST_LIB pointing at it."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]
import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native  # noqa: E402

lib = _native.load()
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(1920, 1080)
sc = gs_scenes.random_gaussians(1_000_000, 3, cam=cam, seed=0).to(dev)
s = gs_scenes.raster_settings_for(cam, 3, device=dev)
dpix = gs_scenes.dl_dimage(1080, 1920).to(dev)
leaves = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
buf = (ctypes.c_ulonglong * 80)()
for it in range(2):
    lib.gs_debug_bwd_stats(buf, 1)
    m2 = torch.zeros_like(leaves[0], requires_grad=True)
    img, radii = GaussianRasterizer(s)(means3D=leaves[0], means2D=m2, opacities=leaves[2], shs=leaves[1],
                                       scales=leaves[3], rotations=leaves[4])
    (img * dpix).sum().backward()
    torch.cuda.synchronize()
lib.gs_debug_bwd_stats(buf, 0)
h = list(buf)
ev, applied = h[65], sum(h[1:65])
print(f"evaluated {ev}  applied {applied} ({applied / ev:.3f})  no-lane {h[0]}  contributing pixels {h[67]}")
print(f"mean active lanes per applied entry {sum(k * h[k] for k in range(65)) / max(applied, 1):.2f}, "
      f"mean contributing pixels per applied entry {h[67] / max(applied, 1):.2f}")
cum = 0
for k in range(1, 65):
    cum += h[k]
    if k in (1, 2, 4, 8, 12, 16, 24, 32, 48, 64):
        print(f"  <= {k:2d} lanes: {cum / applied:.3f}")
