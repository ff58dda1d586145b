"""Debug: the worst image pixel of the large/needle dense comparison and the decisions along its walk."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), os.path.join(ROOT, "tests"), ROOT]
import numpy as np
import torch
import dense_ref, gs_scenes
from diff_gaussian_rasterization import GaussianRasterizer

dev = torch.device("cuda:0")
W, H = 640, 360
cam = gs_scenes.identity_camera(W, H)
small = gs_scenes.random_gaussians(3000, 2, cam=cam, seed=21)
big = gs_scenes.random_gaussians(60, 2, cam=cam, seed=22, scale_range=(0.3, 1.5), z_range=(2.0, 4.0))
big.scales[::3, 0] /= 60.0
d = gs_scenes.concat_scenes(small, big).to(dev)
bg = torch.tensor([0.1, 0.2, 0.3], device=dev)
s = gs_scenes.raster_settings_for(cam, 2, bg=bg, device=dev)
with torch.no_grad():
    img, radii = GaussianRasterizer(s)(means3D=d.means3D, means2D=torch.zeros_like(d.means3D), opacities=d.opacities,
                                       shs=d.shs, scales=d.scales, rotations=d.rotations)
f = torch.float64
args = (d.means3D.to(f), torch.zeros_like(d.means3D, dtype=f), d.opacities.to(f), cam.world_view_transform.to(dev, f),
        cam.full_proj_transform.to(dev, f), cam.camera_center.to(dev, f), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2),
        W, H, bg.to(f))
with torch.no_grad():
    rimg, rradii, flag = dense_ref.render_local(*args, shs=d.shs.to(f), deg=2, scales=d.scales.to(f),
                                                rots=d.rotations.to(f), flag_T_rel=1e-3)
diff = (img.double() - rimg).abs().amax(0)
diff[flag] = 0
y, x = np.unravel_index(int(torch.argmax(diff)), diff.shape)
print("worst pixel", x, y, "diff", float(diff[y, x]), "hip", img[:, y, x].tolist(), "ref", rimg[:, y, x].tolist())
q = dense_ref._prep(*args[:10], shs=d.shs.to(f), deg=2, scales=d.scales.to(f), rots=d.rotations.to(f))
pix, conic, order = q["pix"], q["conic"], q["order"]
x0, y0, x1, y1 = q["x0"], q["y0"], q["x1"], q["y1"]
T = 1.0
for i in order:
    if not (x0[i] <= x // 16 < x1[i] and y0[i] <= y // 16 < y1[i]):
        continue
    dx, dy = float(pix[i, 0]) - x, float(pix[i, 1]) - y
    power = -0.5 * (float(conic[i, 0]) * dx * dx + float(conic[i, 2]) * dy * dy) - float(conic[i, 1]) * dx * dy
    a = min(0.99, float(d.opacities[i]) * math.exp(power))
    if power > 0 or a < 1 / 255:
        if abs(a * 255 - 1) < 1e-2 or abs(power) < 1e-3:
            print(f"  skip near: i {i} power {power:.6e} alpha*255 {a*255:.6f}")
        continue
    tt = T * (1 - a)
    print(f"  i {i} alpha {a:.6f} alpha*255-1 {a*255-1:.3e} T {T:.6e} testT/1e-4-1 {tt/1e-4-1:.3e} big {i >= 3000}")
    if tt < 1e-4:
        print("  stop"); break
    T = tt
