"""Minimal runner for profiling one train.py iteration (gs_train_step.train_step) at C3 under
rocprofv3: W warm-up + K timed iterations, fused glue (default) or the reference's torch glue."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]
import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_train_step as ts  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--torch-glue", action="store_true")
ap.add_argument("--no-split-sh", action="store_true")
ap.add_argument("--loss-item", action="store_true", help="train.py's per-iteration loss.item()")
ap.add_argument("--fuse-adam", action="store_true", help="train_step(fuse_adam=True)")
ap.add_argument("--lr-zero", action="store_true", help="every learning rate 0: the scene stays the C3 scene")
a = ap.parse_args()
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(1920, 1080)
sc = gs_scenes.random_gaussians(1_000_000, 3, cam=cam, seed=0)
settings = gs_scenes.raster_settings_for(cam, 3, device=dev)
gt = torch.rand((3, 1080, 1920), generator=torch.Generator().manual_seed(2)).to(dev)
model = ts.TrainModel(sc, dev, fused=not a.torch_glue)
if a.lr_zero:
    for g in model.optimizer.param_groups:
        g["lr"] = 0.0
for _ in range(a.warmup):
    ts.train_step(model, settings, gt, fused=not a.torch_glue, split_sh=not a.no_split_sh, loss_item=a.loss_item,
                  fuse_adam=a.fuse_adam)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    ts.train_step(model, settings, gt, fused=not a.torch_glue, split_sh=not a.no_split_sh, loss_item=a.loss_item,
                  fuse_adam=a.fuse_adam)
torch.cuda.synchronize()
print(f"train step {1e3 * (time.perf_counter() - t) / a.steps:.3f} ms")
