"""Diagnostic: tests/test_gpu_multiview.py::test_raw_backward_returns_every_upstream_gradient's scene
(3000 Gaussians, SH2, 160x120, exact numerics) through the library named by $GSRAST_LIB, beside the C
oracle (fp64 sums of fp32 per-pixel terms) and the dense fp64 autograd reference (tests/dense_ref.py,
flagged pixels' dL/dpix zeroed for all three).  Prints, per chain gradient, each one's distance to the
dense reference, and the worst elements of the device-vs-oracle difference."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT, os.path.join(ROOT, "tests")]

import dense_ref  # noqa: E402
import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native  # noqa: E402
from oracle import gs_oracle  # noqa: E402

tag = sys.argv[1]
_native.load().gs_set_exact_exp(1)
dev = torch.device("cuda:0")
W, H = 160, 120
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(3000, 2, cam=cam, seed=17)
bgn = np.array([0.1, 0.0, 0.2], np.float32)
bg = torch.tensor(bgn, device=dev)
dpix = gs_scenes.dl_dimage(H, W, seed=18)
leaves = {"means3D": sc.means3D, "opacities": sc.opacities, "shs": sc.shs, "scales": sc.scales,
          "rotations": sc.rotations}
t = {k: v.detach().double().to(dev).clone().requires_grad_(True) for k, v in leaves.items()}
t["means2D"] = torch.zeros_like(t["means3D"], requires_grad=True)
f = torch.float64
rimg, _, flag = dense_ref.render_local(
    t["means3D"], t["means2D"], t["opacities"], cam.world_view_transform.to(dev, f), cam.full_proj_transform.to(dev, f),
    cam.camera_center.to(dev, f), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), W, H, bg.double(), shs=t["shs"],
    deg=2, scales=t["scales"], rots=t["rotations"], flag_rel=1e-4, flag_T_rel=1e-3)
dpm = (dpix.to(dev) * (~flag)[None])
(rimg * dpm.double()).sum().backward()
h = {k: v.detach().to(dev).clone().requires_grad_(True) for k, v in leaves.items()}
m2 = torch.zeros_like(h["means3D"], requires_grad=True)
s = gs_scenes.raster_settings_for(cam, 2, bg=bg, device=dev)
img, _ = GaussianRasterizer(s)(means3D=h["means3D"], means2D=m2, opacities=h["opacities"], shs=h["shs"],
                               scales=h["scales"], rotations=h["rotations"])
(img * dpm).sum().backward()
torch.cuda.synchronize()
osc = gs_oracle.Scene(bg=bgn, means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(), W=W, H=H,
                      viewmatrix=cam.world_view_transform.numpy(), projmatrix=cam.full_proj_transform.numpy(),
                      campos=cam.camera_center.numpy(), tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
                      shs=sc.shs.numpy(), sh_degree=2, scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
gr = gs_oracle.backward(osc, dpm.cpu().numpy())
print(f"{tag}: flagged pixels {int(flag.sum())}")
for k, rk in (("means3D", "dmeans3D"), ("scales", "dscales"), ("rotations", "drotations"), ("opacities", "dopacity")):
    ref = t[k].grad.detach().cpu().numpy()
    g = h[k].grad.detach().cpu().numpy().astype(np.float64)
    o = gr[rk].reshape(g.shape).astype(np.float64)
    sc_ = np.abs(ref).max()
    dg, do, dgo = np.abs(g - ref), np.abs(o - ref), np.abs(g - o)
    w = np.unravel_index(np.argmax(dgo), dgo.shape)
    print(f"{tag} {k}: max|gpu-dense| {dg.max() / sc_:.2e}  max|oracle-dense| {do.max() / sc_:.2e} (of max)  "
          f"worst gpu-vs-oracle {w}: gpu {g[w]:.6e} oracle {o[w]:.6e} dense {ref[w]:.6e}")
