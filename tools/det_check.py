"""Run-to-run determinism check of the rasterizer (fast mode, the C2 parity case): forward +
backward repeated in one process, every output compared bitwise with the first run."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(R, "tests"), os.path.join(R, "gaussian-splatting-skysphere_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

n_runs = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(800, 800)
sc = gs_scenes.random_gaussians(100_000, 3, cam=cam, seed=0)
dpix = gs_scenes.dl_dimage(800, 800, seed=1).to(dev)
s = gs_scenes.raster_settings_for(cam, 3, device=dev)
d = sc.to(dev)


def run():
    leaves = dict(means3D=d.means3D.clone().requires_grad_(True), shs=d.shs.clone().requires_grad_(True),
                  opacities=d.opacities.clone().requires_grad_(True), scales=d.scales.clone().requires_grad_(True),
                  rotations=d.rotations.clone().requires_grad_(True))
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    img, _ = GaussianRasterizer(s)(means2D=means2D, **leaves)
    (img * dpix).sum().backward()
    torch.cuda.synchronize()
    out = {"img": img.detach().clone(), "means2D": means2D.grad.clone()}
    out.update({k: v.grad.clone() for k, v in leaves.items()})
    return out


ref = run()
bad = 0
for r in range(1, n_runs):
    o = run()
    diff = {k: float((o[k] - ref[k]).abs().max()) for k in ref if not torch.equal(o[k], ref[k])}
    if diff:
        bad += 1
        nz = {k: int((o[k] != ref[k]).sum()) for k in diff}
        print(f"run {r}: differs {diff} elements {nz}", flush=True)
print(f"{n_runs} runs, {bad} differing", flush=True)
