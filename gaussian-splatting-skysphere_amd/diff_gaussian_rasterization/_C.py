"""Native entry points of `diff_gaussian_rasterization`, bound to libgsrast.so (C ABI, gfx950).

Same names, argument order, return tuples and error behaviour as the upstream torch extension
`diff_gaussian_rasterization._C` that the reference binds (un-vendored submodule,
/root/reference/.gitmodules:4-6; signatures restated in SURVEY.md §8b):

    rasterize_gaussians(...)           -> (num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer)
    rasterize_gaussians_backward(...)  -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D,
                                           dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)
    mark_visible(means3D, viewmatrix, projmatrix) -> bool[P]

Tensors must live on a HIP device; all work is enqueued on the current torch stream of that
device.  There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

_lib = _native.load()


def _dev_check(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(
            f"diff_gaussian_rasterization (MI355X/HIP) needs device tensors; {name} is on {t.device}. "
            "There is no CPU rasterizer in the product path."
        )


def _f32(t, name, device, allow_empty=True):
    """Contiguous fp32 device tensor, or None for an absent / empty input."""
    if t is None:
        return None
    if t.numel() == 0:
        if allow_empty:
            return None
        raise RuntimeError(f"{name} must not be empty")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    if t.device != device:
        # small camera-side tensors (bg, matrices, campos) may be handed over on the host
        if t.numel() <= 16:
            t = t.to(device)
        else:
            _dev_check(t, name)
            raise RuntimeError(f"{name} is on {t.device}, expected {device}")
    return t.contiguous()


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _Inputs:
    """Validated, contiguous views of one rasterizer call's tensors."""

    def __init__(self, background, means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix,
                 projmatrix, sh, campos, need_opacity=True):
        if means3D.ndimension() != 2 or means3D.size(1) != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        _dev_check(means3D, "means3D")
        self.device = means3D.device
        d = self.device
        self.P = means3D.size(0)
        self.means3D = _f32(means3D, "means3D", d)
        self.bg = _f32(background, "background", d)
        self.colors = _f32(colors, "colors_precomp", d)
        self.opacity = _f32(opacity, "opacities", d)
        self.scales = _f32(scales, "scales", d)
        self.rotations = _f32(rotations, "rotations", d)
        self.cov3D = _f32(cov3D_precomp, "cov3D_precomp", d)
        self.view = _f32(viewmatrix, "viewmatrix", d)
        self.proj = _f32(projmatrix, "projmatrix", d)
        self.sh = _f32(sh, "sh", d)
        self.campos = _f32(campos, "campos", d)
        self.M = 0 if self.sh is None else (self.sh.size(1) if self.sh.ndimension() == 3 else self.sh.numel() // max(1, 3 * self.P))
        if self.P > 0:
            if self.colors is not None and self.colors.numel() != 3 * self.P:
                raise RuntimeError("colors_precomp must have shape (P, 3)")
            if need_opacity and (self.opacity is None or self.opacity.numel() != self.P):
                raise RuntimeError("opacities must have shape (P, 1)")

    def common(self):
        return (_ptr(self.means3D), _ptr(self.sh), _ptr(self.colors), _ptr(self.opacity), _ptr(self.scales))


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug):
    x = _Inputs(background, means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh,
                campos)
    H, W = int(image_height), int(image_width)
    dev = x.device
    u8 = dict(dtype=torch.uint8, device=dev)
    if x.P == 0:
        # upstream: nothing is launched for an empty scene; the image stays all-zero (no background)
        return (0, torch.zeros((3, H, W), dtype=torch.float32, device=dev), torch.zeros((0,), dtype=torch.int32,
                                                                                        device=dev),
                torch.empty((0,), **u8), torch.empty((0,), **u8), torch.empty((0,), **u8))
    # every pixel of the image and every radius is written by the kernels
    out_color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
    radii = torch.empty((x.P,), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        st = _stream(dev)
        geom = torch.empty((_lib.gs_geom_buffer_bytes(x.P),), **u8)
        nr = ctypes.c_longlong(0)
        _native.check(
            _lib.gs_forward_preprocess(
                x.P, int(degree), x.M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh), _ptr(x.colors),
                _ptr(x.opacity), _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D),
                _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy), int(bool(prefiltered)),
                _ptr(radii), _ptr(geom), ctypes.byref(nr), int(bool(debug)), st),
            "rasterize_gaussians (preprocess)")
        num_rendered = int(nr.value)
        binning = torch.empty((_lib.gs_binning_buffer_bytes(num_rendered, W, H),), **u8)
        img = torch.empty((_lib.gs_image_buffer_bytes(W, H),), **u8)
        _native.check(
            _lib.gs_forward_render(
                x.P, _ptr(x.bg), W, H, _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy),
                _ptr(radii), _ptr(geom), num_rendered, _ptr(binning), _ptr(img), _ptr(out_color),
                int(bool(debug)), st),
            "rasterize_gaussians (render)")
    return num_rendered, out_color, radii, geom, binning, img


def backward_impl(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                  projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer, R, binningBuffer,
                  imageBuffer, debug, want_all=True):
    """Shared backward.  With want_all=False the gradients that no autograd input can receive
    (colours when SHs drive the colour, cov3D when scale/rotation drive it, ...) are None and
    not computed."""
    x = _Inputs(background, means3D, colors, None, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh,
                campos, need_opacity=False)
    P, dev = x.P, x.device
    f32 = dict(dtype=torch.float32, device=dev)
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = x.M
    need_col = want_all or x.colors is not None
    need_cov = want_all or x.cov3D is not None
    need_sh = want_all or x.sh is not None
    need_sr = want_all or (x.scales is not None and x.rotations is not None)
    dmeans2D = torch.empty((P, 3), **f32)
    dopacity = torch.empty((P, 1), **f32)
    dmeans3D = torch.empty((P, 3), **f32)
    dcolors = (torch.empty if x.colors is not None else torch.zeros)((P, 3), **f32) if need_col else None
    dcov3D = (torch.empty if x.cov3D is not None else torch.zeros)((P, 6), **f32) if need_cov else None
    dsh = (torch.empty if x.sh is not None else torch.zeros)((P, M, 3), **f32) if need_sh else None
    has_sr = x.scales is not None and x.rotations is not None and x.cov3D is None
    dscales = (torch.empty if has_sr else torch.zeros)((P, 3), **f32) if need_sr else None
    drot = (torch.empty if has_sr else torch.zeros)((P, 4), **f32) if need_sr else None
    if P == 0:
        return dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot
    dpix = _f32(dL_dout_color, "dL_dout_color", dev)
    with torch.cuda.device(dev):
        st = _stream(dev)
        grad_scratch = torch.empty((_lib.gs_grad_buffer_bytes(int(R)),), dtype=torch.uint8, device=dev)
        _native.check(
            _lib.gs_backward(
                P, int(degree), M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh), _ptr(x.colors), _ptr(x.opacity),
                _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D), _ptr(x.view), _ptr(x.proj),
                _ptr(x.campos), float(tan_fovx), float(tan_fovy), _ptr(radii), _ptr(geomBuffer), int(R),
                _ptr(binningBuffer), _ptr(imageBuffer), _ptr(dpix), _ptr(grad_scratch), _ptr(dmeans2D),
                _ptr(dcolors if x.colors is not None or need_col else None), _ptr(dopacity), _ptr(dmeans3D),
                _ptr(dcov3D if x.cov3D is not None else None), _ptr(dsh if x.sh is not None else None),
                _ptr(dscales if has_sr else None), _ptr(drot if has_sr else None), int(bool(debug)), st),
            "rasterize_gaussians_backward")
    return dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh,
                                 degree, campos, geomBuffer, R, binningBuffer, imageBuffer, debug):
    return backward_impl(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp,
                         viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer,
                         R, binningBuffer, imageBuffer, debug, want_all=True)


def mark_visible(means3D, viewmatrix, projmatrix):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _dev_check(means3D, "means3D")
    dev = means3D.device
    P = means3D.size(0)
    present = torch.zeros((P,), dtype=torch.bool, device=dev)
    if P == 0:
        return present
    m = _f32(means3D, "means3D", dev)
    v = _f32(viewmatrix, "viewmatrix", dev)
    p = _f32(projmatrix, "projmatrix", dev)
    with torch.cuda.device(dev):
        _native.check(_lib.gs_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(dev)), "mark_visible")
    return present


def debug_export(P, W, H, num_rendered, geomBuffer, binningBuffer, imageBuffer, device):
    """Forward intermediates for tests: dict of device tensors."""
    u32 = dict(dtype=torch.int32, device=device)
    f32 = dict(dtype=torch.float32, device=device)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    out = dict(
        point_list=torch.zeros((max(num_rendered, 1),), **u32),
        ranges=torch.zeros((gx * gy, 2), **u32),
        xy=torch.zeros((P, 2), **f32),
        conic_opacity=torch.zeros((P, 4), **f32),
        rgb=torch.zeros((P, 3), **f32),
        depth=torch.zeros((P,), **f32),
        tiles_touched=torch.zeros((P,), **u32),
        final_T=torch.zeros((H, W), **f32),
        n_contrib=torch.zeros((H, W), **u32),
    )
    if P > 0:
        with torch.cuda.device(device):
            _native.check(
                _lib.gs_debug_export(P, W, H, int(num_rendered), _ptr(geomBuffer), _ptr(binningBuffer),
                                     _ptr(imageBuffer), *[_ptr(out[k]) for k in (
                                         "point_list", "ranges", "xy", "conic_opacity", "rgb", "depth",
                                         "tiles_touched", "final_T", "n_contrib")], _stream(device)),
                "debug_export")
    out["point_list"] = out["point_list"][:num_rendered]
    return out
