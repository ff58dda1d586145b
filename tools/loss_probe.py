"""The fused photometric loss (gs_loss.photometric_loss, train.py:91-92) alone at 3x1080x1920:
forward + backward in a loop, for rocprofv3 kernel traces / PMC passes of k_ssim_fwd / k_ssim_bwd
(tools/pmc_ab.sh-style: --kernel-include-regex ssim).  Prints the mean ms per iteration."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]
import torch  # noqa: E402

import gs_loss  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--warmup", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
img = torch.rand((3, 1080, 1920), generator=g).to(dev).requires_grad_(True)
gt = torch.rand((3, 1080, 1920), generator=g).to(dev)


def step():
    img.grad = None
    loss, _ = gs_loss.photometric_loss(img, gt)
    loss.backward()


for _ in range(a.warmup):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
print(json.dumps({"loss_fwd_bwd_ms": round((time.perf_counter() - t) / a.steps * 1e3, 4)}))
