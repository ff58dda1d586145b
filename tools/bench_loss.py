"""Photometric loss of train.py:91-92 at 1080p on one GPU: the reference formulation (five
depthwise conv2d + autograd, restated from utils/loss_utils.py in torch fp32) vs the fused HIP
SSIM (gs_loss).  Prints one JSON line."""
import json
import os
import sys
import time
from math import exp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import gs_loss  # noqa: E402


def ref_ssim(img1, img2):
    """torch fp32 restatement of /root/reference/utils/loss_utils.py:_ssim (the reference's path)."""
    g = torch.tensor([exp(-(x - 5) ** 2 / float(2 * 1.5 ** 2)) for x in range(11)])
    g = g / g.sum()
    w = (g[:, None] @ g[None, :]).float()[None, None].expand(3, 1, 11, 11).contiguous().to(img1.device)
    c = lambda t: F.conv2d(t, w, padding=5, groups=3)  # noqa: E731
    mu1, mu2 = c(img1), c(img2)
    m11, m22, m12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1, s2, s12 = c(img1 * img1) - m11, c(img2 * img2) - m22, c(img1 * img2) - m12
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    return (((2 * m12 + C1) * (2 * s12 + C2)) / ((m11 + m22 + C1) * (s1 + s2 + C2))).mean()


def timeit(fn, steps=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
img = torch.rand((3, 1080, 1920), generator=g).to(dev).requires_grad_(True)
gt = torch.rand((3, 1080, 1920), generator=g).to(dev)
lam = 0.2


def step(ssim_fn):
    def f():
        img.grad = None
        loss = (1.0 - lam) * gs_loss.l1_loss(img, gt) + lam * (1.0 - ssim_fn(img, gt))
        loss.backward()
    return f


t_ref = timeit(step(ref_ssim))
t_fused = timeit(step(gs_loss.ssim))
print(json.dumps({"workload": "train.py:91-92 loss fwd+bwd, 3x1080x1920 fp32", "ref_conv2d_ms": round(t_ref, 4),
                  "fused_ms": round(t_fused, 4), "speedup": round(t_ref / t_fused, 2)}))
