"""Diagnostic: the dense-reference needle scene of tests/test_gpu_dense.py through the HIP path of the
library named by $GSRAST_LIB, plus the fp64 dense reference; saves every gradient to
gpurun_out/dense_diag_<tag>.npz for an offline comparison of library builds."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT, os.path.join(ROOT, "tests")]

import dense_ref  # noqa: E402
import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

tag = sys.argv[1]
dev = torch.device("cuda:0")
W, H = 640, 360
cam = gs_scenes.identity_camera(W, H)
small = gs_scenes.random_gaussians(3000, 2, cam=cam, seed=21)
big = gs_scenes.random_gaussians(60, 2, cam=cam, seed=22, scale_range=(0.3, 1.5), z_range=(2.0, 4.0))
big.scales[::3, 0] /= 60.0
d = gs_scenes.concat_scenes(small, big).to(dev)
leaves = {k: getattr(d, k) for k in ("means3D", "opacities", "shs", "scales", "rotations")}
leaves["means2D"] = torch.zeros_like(d.means3D)
bg = torch.tensor([0.1, 0.2, 0.3], device=dev)
dpix = gs_scenes.dl_dimage(H, W, seed=24, scale=1.0).to(dev)
s = gs_scenes.raster_settings_for(cam, 2, bg=bg, device=dev)
hip = {k: v.detach().clone().requires_grad_(True) for k, v in leaves.items()}
img, radii = GaussianRasterizer(s)(means3D=hip["means3D"], means2D=hip["means2D"], opacities=hip["opacities"],
                                   shs=hip["shs"], scales=hip["scales"], rotations=hip["rotations"])
t = {k: v.detach().double().clone().requires_grad_(True) for k, v in leaves.items()}
f = torch.float64
rimg, rradii, flag = dense_ref.render_local(
    t["means3D"], t["means2D"], t["opacities"], cam.world_view_transform.to(dev, f), cam.full_proj_transform.to(dev, f),
    cam.camera_center.to(dev, f), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), W, H, bg.double(), shs=t["shs"],
    deg=2, scales=t["scales"], rots=t["rotations"], flag_rel=2e-4, flag_T_rel=1e-3)
dpm = dpix * (~flag)[None]
(img * dpm).sum().backward()
(rimg * dpm.double()).sum().backward()
torch.cuda.synchronize()
out = {}
for k in hip:
    out["hip_" + k] = hip[k].grad.detach().cpu().numpy()
    out["ref_" + k] = t[k].grad.detach().cpu().numpy()
out["img"] = img.detach().cpu().numpy()
out["flag"] = flag.cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"dense_diag_{tag}.npz"), **out)
for k in hip:
    a, r = out["hip_" + k].astype(np.float64), out["ref_" + k]
    dd = np.abs(a - r).reshape(len(a), -1).max(1)
    top = np.argsort(-dd)[:5]
    print(f"{tag} d{k}: max|d| {dd.max():.3e} max|ref| {np.abs(r).max():.3e} worst {list(top)} {[f'{x:.2e}' for x in dd[top]]}")
