"""Why does k_render_bwd_tw run longer inside the train step than in the bench loop?

C3 batch-1 iterations (one view's forward + full backward into a GradBucket, one stream), with
what runs between the forward and the backward varied; render_bwd (and render_fwd, preprocess_bwd)
from the library's HIP-event profile:
  plain      forward -> backward(dL/dpix fixed)                     (the bench's single_view loop)
  loss       forward -> photometric loss fwd + bwd -> backward(dL/dimage of that loss)  (train.py)
  loss_fix   forward -> photometric loss fwd + bwd -> backward(the fixed dL/dpix): the loss kernels'
             cache footprint without their dL/dimage values
  flush      forward -> a 512 MB fill (evicts L2 and the 256 MB MALL) -> backward(fixed dL/dpix)
  tiny       forward -> backward(the fixed dL/dpix times 1e-6, the magnitude of the loss's
             dL/dimage): the values' effect alone
Rounds alternate the modes; prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_loss  # noqa: E402
import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native  # noqa: E402

P, deg, W, H = 1_000_000, 3, 1920, 1080
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
bucket = vp.GradBucket(params, lazy_zero=True, defer=False)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(5)).to(dev)
flush = torch.empty((512 << 20) // 4, dtype=torch.float32, device=dev)
r = GaussianRasterizer(gs_scenes.raster_settings_for(cam, deg, device=dev))


def step(mode):
    bucket.zero_grad()
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4])
    if mode in ("loss", "loss_fix"):
        loss, _ = gs_loss.photometric_loss(img, gt)
        if mode == "loss":
            loss.backward()
        else:
            g = torch.autograd.grad(loss, img)[0]
            img.backward(dpix + 0 * g[:1, :1, :1])
    elif mode == "flush":
        flush.fill_(1.0)
        img.backward(dpix)
    elif mode == "tiny":
        img.backward(dpix * 1e-6)
    else:
        img.backward(dpix)
    bucket.finalize()


modes = ["plain", "loss", "loss_fix", "flush", "tiny"]
lib = _native.load()
res = {m: [] for m in modes}
for m in modes:
    for _ in range(5):
        step(m)
torch.cuda.synchronize()
for rnd in range(3):
    for m in modes:
        lib.gs_profile_reset()
        lib.gs_profile_enable(1)
        for _ in range(30):
            step(m)
        torch.cuda.synchronize()
        lib.gs_profile_enable(0)
        prof = _native.profile_stats()
        res[m].append({k: round(1e3 * ms / max(n, 1), 2) for k, (ms, n) in prof.items()
                       if k in ("render_bwd", "render_fwd", "preprocess_bwd", "sum_records", "tile_order")})
print(json.dumps({"workload": "c3 batch 1", "iters_per_round": 30, "rounds": res}))

# The train step itself (gs_train_step.train_step, fused Adam, loss.item()), with the optimizer's
# learning rates as train.py sets them and all set to 0 (the scene then stays the C3 scene): the
# render kernels' times and the instance count after each block of iterations.
import gs_train_step as ts  # noqa: E402
from diff_gaussian_rasterization import last_num_rendered  # noqa: E402

settings = gs_scenes.raster_settings_for(cam, deg, device=dev)
out = {}
for lr_on in (True, False):
    m = ts.TrainModel(gs_scenes.random_gaussians(P, deg, cam=cam, seed=0), dev)
    if not lr_on:
        for g_ in m.optimizer.param_groups:
            g_["lr"] = 0.0
    blocks = []
    for blk in range(4):
        lib.gs_profile_reset()
        lib.gs_profile_enable(1)
        for _ in range(10):
            ts.train_step(m, settings, gt, loss_item=True, fuse_adam=True)
        torch.cuda.synchronize()
        lib.gs_profile_enable(0)
        prof = _native.profile_stats()
        blocks.append({"iters": 10 * (blk + 1), "num_rendered": last_num_rendered(),
                       **{k: round(1e3 * ms / max(n, 1), 2) for k, (ms, n) in prof.items()
                          if k in ("render_bwd", "render_fwd")}})
    out["lr_train_py" if lr_on else "lr_zero"] = blocks
    del m
print(json.dumps({"train_step": out}))
