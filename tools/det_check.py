"""Run-to-run determinism check of the rasterizer (fast mode): forward + backward repeated in one
process, every output compared bitwise with the first run.  Usage: det_check.py [runs] [c2|c3] [alt]
(alt: every other run uses a second dL/dimage and a second scene in between, so the scratch buffers
the caching allocator hands back hold the other run's data -- stale reads show up as differences)."""
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
big = len(sys.argv) > 2 and sys.argv[2] == "c3"
alt = len(sys.argv) > 3 and sys.argv[3] == "alt"
dev = torch.device("cuda:0")
W, H, P = (1920, 1080, 1_000_000) if big else (800, 800, 100_000)
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, 3, cam=cam, seed=0)
dpix = gs_scenes.dl_dimage(H, W, seed=1).to(dev)
dpix2 = gs_scenes.dl_dimage(H, W, seed=2).to(dev)
s = gs_scenes.raster_settings_for(cam, 3, device=dev)
d = sc.to(dev)
sc2 = gs_scenes.random_gaussians(P, 3, cam=cam, seed=5).to(dev)


def run(d=d, dpix=dpix):
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
    if alt:
        run(sc2, dpix2)
        run(d, dpix2)
    o = run()
    diff = {k: float((o[k] - ref[k]).abs().max()) for k in ref if not torch.equal(o[k], ref[k])}
    if diff:
        bad += 1
        nz = {k: int((o[k] != ref[k]).sum()) for k in diff}
        print(f"run {r}: differs {diff} elements {nz}", flush=True)
print(f"{n_runs} runs, {bad} differing", flush=True)
