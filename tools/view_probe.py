"""Is render_fwd slower in bench.py's 4-view step (≈ 175 µs per launch) than in the batch-1 loop
(≈ 164 µs) because of the views or because of the step?  C3: each of the step's four jittered
cameras (bench.py's rank 0, seed 7) run alone as a batch-1 loop, then the 4-view step on one stream
(prepared views, deferred per-Gaussian pass) as bench.py's event pass runs it; render_fwd / render_bwd
per launch from the library's HIP-event profile, plus each view's walked instances."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native, prepare_views  # noqa: E402

P, deg, W, H = 1_000_000, 3, 1920, 1080
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
cams = gs_scenes.jittered_cameras(4, W, H, seed=7)
cams[0] = cam
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
dpix = gs_scenes.dl_dimage(H, W, seed=1).to(dev)
rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, deg, device=dev)) for c in cams]
lib = _native.load()


def prof(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    lib.gs_profile_reset()
    lib.gs_profile_enable(1)
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    lib.gs_profile_enable(0)
    return {k: round(1e3 * ms / max(c, 1), 2) for k, (ms, c) in _native.profile_stats().items()
            if k in ("render_fwd", "render_bwd", "sum_records")}


out = {"single": []}
b1 = vp.GradBucket(params, lazy_zero=True, defer=False)
for v, r in enumerate(rasts):
    def step(r=r):
        b1.zero_grad()
        m2 = torch.empty_like(params[0], requires_grad=True)
        img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                   rotations=params[4])
        img.backward(dpix)
        b1.finalize()
    out["single"].append({"view": v, **prof(step, 30)})
b1.close()
b4 = vp.GradBucket(params, lazy_zero=True, defer=True)
st = [torch.cuda.current_stream(dev)]


def step4():
    b4.zero_grad()
    pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4], streams=st * 4)
    for r, p in zip(rasts, pre):
        m2 = torch.empty_like(params[0], requires_grad=True)
        img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                   rotations=params[4], prepared=p)
        img.backward(dpix)
    b4.finalize()


out["step4_one_stream"] = prof(step4, 20)
print(json.dumps(out))
