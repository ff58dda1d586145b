"""Photometric loss of train.py on MI355X: drop-in `l1_loss` / `ssim` for utils.loss_utils.

The reference computes `loss = (1 - lambda) * l1_loss(image, gt) + lambda * (1 - ssim(image, gt))`
every iteration (/root/reference/train.py:91-92) with five depthwise conv2d calls and their
autograd backward (/root/reference/utils/loss_utils.py:33-60).  `ssim` here is one fused HIP
forward (separable 11-tap window through LDS, SSIM map sum, per-pixel partials) and one fused
backward (csrc/gs_loss.hip, C ABI gs_ssim_forward / gs_ssim_backward).  Same signature, same
value (fp32), same gradient w.r.t. the rendered image; the target image gets no gradient (as in
train.py, where it is data).  Use:  `from gs_loss import l1_loss, ssim`.

`photometric_loss(image, gt, lambda_dssim)` is the whole expression of train.py:91-92 fused
(SURVEY.md §8f row 4): the SSIM kernel also sums |image - gt| per tile, one fixed-order reduction
forms `(1 - lambda) L1 + lambda (1 - SSIM)` on the device, and one backward kernel writes both
terms' gradient -- no elementwise / reduction kernels of torch around it.  It returns the loss and
the L1 term (detached, for the reference's logging of Ll1, train.py:100).
"""
from __future__ import annotations

import ctypes
from math import exp

import torch

from diff_gaussian_rasterization import _native

_lib = _native.load()


def _window11() -> ctypes.Array:
    # loss_utils.gaussian(11, 1.5): float32 tensor of Python-double exps, divided by its sum
    g = torch.tensor([exp(-(x - 5) ** 2 / float(2 * 1.5 ** 2)) for x in range(11)], dtype=torch.float32)
    g = g / g.sum()
    return (ctypes.c_float * 11)(*g.tolist())


_WIN = _window11()
_WIN_P = ctypes.cast(_WIN, ctypes.c_void_p)


def l1_loss(network_output, gt):
    """utils/loss_utils.py:17-18 (a single fused elementwise mean in torch already)."""
    return torch.abs((network_output - gt)).mean()


def _planes(img):
    if img.dim() == 3:
        return 1, img.shape[0], img.shape[1], img.shape[2]
    if img.dim() == 4:
        return img.shape[0], img.shape[1], img.shape[2], img.shape[3]
    raise ValueError("ssim expects [C, H, W] or [B, C, H, W] images")


class _SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img1, img2, size_average):
        if not img1.is_cuda:
            raise RuntimeError("gs_loss.ssim (MI355X/HIP) needs device tensors; there is no CPU path")
        if img1.shape != img2.shape:
            raise ValueError(f"ssim: shapes differ {tuple(img1.shape)} vs {tuple(img2.shape)}")
        B, C, H, W = _planes(img1)
        if not size_average and img1.dim() == 3:
            raise ValueError("size_average=False needs [B, C, H, W] images (as in the reference)")
        a = img1.detach().to(torch.float32).contiguous()
        b = img2.detach().to(device=a.device, dtype=torch.float32).contiguous()
        planes = B * C
        dev = a.device
        dmaps = torch.empty((3, planes, H, W), dtype=torch.float32, device=dev)
        partial = torch.empty((_lib.gs_ssim_partial_count(planes, H, W),), dtype=torch.float32, device=dev)
        plane_sum = torch.empty((planes,), dtype=torch.float32, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        with torch.cuda.device(dev):
            _native.check(_lib.gs_ssim_forward(planes, H, W, _WIN_P, ctypes.c_void_p(a.data_ptr()),
                                               ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(dmaps.data_ptr()),
                                               ctypes.c_void_p(partial.data_ptr()),
                                               ctypes.c_void_p(plane_sum.data_ptr()), st), "ssim forward")
        per_image = plane_sum.view(B, C).sum(1) / float(C * H * W)
        out = per_image.mean() if size_average else per_image
        ctx.save_for_backward(a, b, dmaps)
        ctx.shape = (B, C, H, W, size_average, img1.dtype)
        return out.to(img1.dtype)

    @staticmethod
    def backward(ctx, grad):
        a, b, dmaps = ctx.saved_tensors
        B, C, H, W, size_average, dtype = ctx.shape
        if grad is None:
            return None, None, None
        g = grad.to(torch.float32)
        scale = (g.expand(B) / float(B * C * H * W) if size_average else g / float(C * H * W)).contiguous()
        dimg = torch.empty_like(a)
        st = ctypes.c_void_p(torch.cuda.current_stream(a.device).cuda_stream)
        with torch.cuda.device(a.device):
            _native.check(_lib.gs_ssim_backward(B * C, C, H, W, _WIN_P, ctypes.c_void_p(a.data_ptr()),
                                                ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(dmaps.data_ptr()),
                                                ctypes.c_void_p(scale.data_ptr()), ctypes.c_void_p(dimg.data_ptr()),
                                                st), "ssim backward")
        return dimg.to(dtype), None, None


def ssim(img1, img2, window_size=11, size_average=True):
    """utils/loss_utils.py:33-40 (window 11 only, as train.py uses it)."""
    if window_size != 11:
        raise NotImplementedError("gs_loss.ssim implements the 11x11 window of the reference")
    if img2.requires_grad:
        raise NotImplementedError("gs_loss.ssim differentiates w.r.t. img1 only (img2 is the target)")
    return _SSIM.apply(img1, img2, size_average)


class _PhotometricLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, lambda_dssim):
        if not image.is_cuda:
            raise RuntimeError("gs_loss.photometric_loss (MI355X/HIP) needs device tensors; there is no CPU path")
        if image.shape != gt.shape:
            raise ValueError(f"photometric_loss: shapes differ {tuple(image.shape)} vs {tuple(gt.shape)}")
        B, C, H, W = _planes(image)
        a = image.detach().to(torch.float32).contiguous()
        b = gt.detach().to(device=a.device, dtype=torch.float32).contiguous()
        planes = B * C
        dev = a.device
        dmaps = torch.empty((3, planes, H, W), dtype=torch.float32, device=dev)
        partial = torch.empty((2 * _lib.gs_ssim_partial_count(planes, H, W),), dtype=torch.float32, device=dev)
        out = torch.empty((3,), dtype=torch.float32, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        with torch.cuda.device(dev):
            _native.check(_lib.gs_photometric_loss_forward(
                planes, H, W, _WIN_P, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                float(lambda_dssim), ctypes.c_void_p(dmaps.data_ptr()), ctypes.c_void_p(partial.data_ptr()),
                ctypes.c_void_p(out.data_ptr()), st), "photometric loss forward")
        ctx.save_for_backward(a, b, dmaps)
        ctx.lam = float(lambda_dssim)
        ctx.dtype = image.dtype
        loss, l1 = out[0].to(image.dtype), out[1].to(image.dtype)
        ctx.mark_non_differentiable(l1)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the L1 output
        return loss, l1

    @staticmethod
    def backward(ctx, grad, _grad_l1):
        a, b, dmaps = ctx.saved_tensors
        if grad is None:
            return None, None, None
        planes, H, W = dmaps.shape[1], dmaps.shape[2], dmaps.shape[3]
        g = grad.to(torch.float32).reshape(1).contiguous()
        dimg = torch.empty_like(a)
        st = ctypes.c_void_p(torch.cuda.current_stream(a.device).cuda_stream)
        with torch.cuda.device(a.device):
            _native.check(_lib.gs_photometric_loss_backward(
                planes, H, W, _WIN_P, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                ctypes.c_void_p(dmaps.data_ptr()), ctx.lam, ctypes.c_void_p(g.data_ptr()),
                ctypes.c_void_p(dimg.data_ptr()), st), "photometric loss backward")
        return dimg.to(ctx.dtype), None, None


def photometric_loss(image, gt, lambda_dssim=0.2):
    """train.py:91-92 in one fused forward and one fused backward: returns (loss, Ll1) with
    loss = (1 - lambda_dssim) * l1_loss(image, gt) + lambda_dssim * (1 - ssim(image, gt)).
    Ll1 carries no gradient (the reference only logs it)."""
    if gt.requires_grad:
        raise NotImplementedError("gs_loss.photometric_loss differentiates w.r.t. the image only (gt is data)")
    loss, l1 = _PhotometricLoss.apply(image, gt, lambda_dssim)
    return loss, l1.detach()
