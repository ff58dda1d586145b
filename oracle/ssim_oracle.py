"""CPU restatement of the reference photometric loss -- TEST INFRASTRUCTURE ONLY.

Follows /root/reference/utils/loss_utils.py:17-60 (l1_loss; gaussian(11, 1.5) window; _ssim with
five zero-padded depthwise conv2d, C1 = 0.01^2, C2 = 0.03^2; mean of the SSIM map) in float64,
differentiated by autograd.  Pinned against tests/golden/loss_golden.npz (values and gradients
produced by the reference code itself).  Only tests/ import this module.
"""
from __future__ import annotations

from math import exp

import torch
import torch.nn.functional as F


def window1d(size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    g = torch.tensor([exp(-(x - size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(size)],
                     dtype=torch.float32)
    return g / g.sum()


def ssim(img1: torch.Tensor, img2: torch.Tensor, size_average: bool = True, size: int = 11):
    """float64 SSIM with autograd (img1 may require grad)."""
    squeeze = img1.dim() == 3
    x = img1.double()
    y = img2.double()
    if squeeze:
        x, y = x[None], y[None]
    C = x.shape[1]
    w1 = window1d(size).double()
    w = (w1[:, None] @ w1[None, :]).expand(C, 1, size, size).contiguous()
    pad = size // 2
    conv = lambda t: F.conv2d(t, w, padding=pad, groups=C)  # noqa: E731
    mu1, mu2 = conv(x), conv(y)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s1 = conv(x * x) - mu1_sq
    s2 = conv(y * y) - mu2_sq
    s12 = conv(x * y) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    if size_average:
        return m.mean()
    return m.mean(1).mean(1).mean(1)


def l1_loss(a: torch.Tensor, b: torch.Tensor):
    return torch.abs(a.double() - b.double()).mean()
