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
import math
import os

import torch

from . import _native

_lib = _native.load()


def _load_ext():
    """The torch C++ host fast path (_gs_ext, csrc/gs_torch_ext.cpp) of the plain forward / backward
    calls, if built (setup_ext.py); GSRAST_NO_EXT=1 keeps every call on the ctypes path."""
    if os.environ.get("GSRAST_NO_EXT", "0") not in ("", "0"):
        return None
    try:
        from . import _gs_ext
    except ImportError:
        return None
    _gs_ext.init()
    return _gs_ext


_EXT = _load_ext()


def _dev_check(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(
            f"diff_gaussian_rasterization (MI355X/HIP) needs device tensors; {name} is on {t.device}. "
            "There is no CPU rasterizer in the product path."
        )


def _f32(t, name, device, allow_empty=True, host_ok=False):
    """Contiguous fp32 device tensor, or None for an absent / empty input.  host_ok: a camera-side
    input (bg, viewmatrix, projmatrix, campos) may come from the host and is copied over; every
    per-Gaussian tensor must already live on means3D's device."""
    if t is None:
        return None
    if t.numel() == 0:
        if allow_empty:
            return None
        raise RuntimeError(f"{name} must not be empty")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    if t.device != device:
        if host_ok and t.numel() <= 16:
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
                 projmatrix, sh, campos, need_opacity=True, sh_rest=None):
        if means3D.ndimension() != 2 or means3D.size(1) != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        _dev_check(means3D, "means3D")
        self.device = means3D.device
        d = self.device
        self.P = means3D.size(0)
        self.means3D = _f32(means3D, "means3D", d)
        self.bg = _f32(background, "background", d, host_ok=True)
        self.colors = _f32(colors, "colors_precomp", d)
        self.opacity = _f32(opacity, "opacities", d)
        self.scales = _f32(scales, "scales", d)
        self.rotations = _f32(rotations, "rotations", d)
        self.cov3D = _f32(cov3D_precomp, "cov3D_precomp", d)
        self.view = _f32(viewmatrix, "viewmatrix", d, host_ok=True)
        self.proj = _f32(projmatrix, "projmatrix", d, host_ok=True)
        self.sh = _f32(sh, "sh", d)
        self.campos = _f32(campos, "campos", d, host_ok=True)
        self.M = 0 if self.sh is None else (self.sh.size(1) if self.sh.ndimension() == 3 else self.sh.numel() // max(1, 3 * self.P))
        # split SH rows (ABI v8): sh is features_dc [P, 1, 3], sh_rest features_rest [P, M - 1, 3]
        self.sh_rest = _f32(sh_rest, "features_rest", d)
        if self.sh_rest is not None:
            if self.sh is None or self.colors is not None:
                raise RuntimeError("split SH: features_dc and features_rest replace shs (no colors_precomp)")
            if tuple(self.sh.shape) != (self.P, 1, 3) or self.sh_rest.ndimension() != 3 or tuple(
                    self.sh_rest.shape[::2]) != (self.P, 3):
                raise RuntimeError("split SH: expected features_dc [P, 1, 3] and features_rest [P, M - 1, 3]")
            self.M = 1 + self.sh_rest.size(1)
        if self.P > 0:
            if self.colors is not None and self.colors.numel() != 3 * self.P:
                raise RuntimeError("colors_precomp must have shape (P, 3)")
            if need_opacity and (self.opacity is None or self.opacity.numel() != self.P):
                raise RuntimeError("opacities must have shape (P, 1)")

    def common(self):
        return (_ptr(self.means3D), _ptr(self.sh), _ptr(self.colors), _ptr(self.opacity), _ptr(self.scales))


def preprocess_views(backgrounds, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                     viewmatrices, projmatrices, tan_fovx, tan_fovy, image_heights, image_widths, sh, degree, campos,
                     prefiltered, debug, streams=None, capacities=None):
    """First half of K views' forwards in one preprocess launch (gs_forward_preprocess_views):
    returns [(num_rendered, radii, geomBuffer, bounded)] per view, each what rasterize_gaussians
    computes for that camera before its binning; view k's depth ordering is enqueued on streams[k]
    (default: the current stream).  Pass each view's tuple to rasterize_gaussians(..., prepared=).
    capacities: K binning capacities -- nothing is read back (gs_forward_preprocess_views_bounded),
    num_rendered is the capacity and the view's render is bounded (gs_forward_render_bounded)."""
    K = len(viewmatrices)
    if not 1 <= K <= 8:
        raise RuntimeError("preprocess_views: 1 to 8 views per call")
    if _EXT is not None and means3D.is_cuda:
        return list(_EXT.preprocess_views(
            list(backgrounds), means3D, colors, opacity, scales, rotations, float(scale_modifier), cov3D_precomp,
            list(viewmatrices), list(projmatrices), [float(t) for t in tan_fovx], [float(t) for t in tan_fovy],
            [int(h) for h in image_heights], [int(w) for w in image_widths], sh, int(degree), list(campos),
            bool(prefiltered), bool(debug), [s.cuda_stream for s in streams] if streams is not None else [],
            None if capacities is None else [int(c) for c in capacities]))
    xs = [_Inputs(backgrounds[k], means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrices[k],
                  projmatrices[k], sh, campos[k]) for k in range(K)]
    x, dev = xs[0], xs[0].device
    u8 = dict(dtype=torch.uint8, device=dev)
    radii = [torch.empty((x.P,), dtype=torch.int32, device=dev) for _ in range(K)]
    # the views' geometry buffers are slices of one allocation (one stride apart): the library then
    # runs the K depth sorts as one set of launches
    gb = _lib.gs_geom_buffer_bytes(x.P) if x.P else 0
    geom_all = torch.empty((K * gb,), **u8)
    geoms = [geom_all[k * gb:(k + 1) * gb] for k in range(K)]
    if x.P == 0:
        return [(0, r, g, False) for r, g in zip(radii, geoms)]
    if capacities is not None and len(capacities) != K:
        raise RuntimeError("preprocess_views: one capacity per view")
    arr = lambda ts: (ctypes.c_void_p * K)(*[t.data_ptr() if t is not None else None for t in ts])  # noqa: E731
    nr = (ctypes.c_longlong * K)()
    vst = None
    if streams is not None:
        vst = (ctypes.c_void_p * K)(*[s.cuda_stream for s in streams])
    if capacities is not None:
        for k, c in enumerate(capacities):
            nr[k] = int(c)
    with torch.cuda.device(dev):
        _native.check(
            (_lib.gs_forward_preprocess_views if capacities is None else _lib.gs_forward_preprocess_views_bounded)(
                K, x.P, int(degree), x.M, arr([y.bg for y in xs]), (ctypes.c_int * K)(*[int(w) for w in image_widths]),
                (ctypes.c_int * K)(*[int(h) for h in image_heights]), _ptr(x.means3D), _ptr(x.sh), _ptr(x.colors),
                _ptr(x.opacity), _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D),
                arr([y.view for y in xs]), arr([y.proj for y in xs]), arr([y.campos for y in xs]),
                (ctypes.c_float * K)(*[float(t) for t in tan_fovx]), (ctypes.c_float * K)(*[float(t) for t in tan_fovy]),
                int(bool(prefiltered)), arr(radii), arr(geoms), nr, int(bool(debug)), _stream(dev), vst),
            "preprocess_views")
    bounded = capacities is not None
    out = [(int(nr[k]), radii[k], geoms[k], bounded) for k in range(K)]
    W0, H0 = int(image_widths[0]), int(image_heights[0])
    if os.environ.get("GSRAST_BATCH_VIEWS", "1") != "0" and all(
            int(w) == W0 and int(h) == H0 for w, h in zip(image_widths, image_heights)):
        # the K views' binning (duplicate, tile sort, ranges) as one set of launches: every binning
        # buffer is a slice of one allocation, sized for the largest count, which then stands for
        # every view's num_rendered (buffer layout, backward scratch)
        I = max(int(nr[k]) for k in range(K))
        bb, ib = _lib.gs_binning_buffer_bytes(I, W0, H0), _lib.gs_image_buffer_bytes(W0, H0)
        bin_all, img_all = torch.empty((K * bb,), **u8), torch.empty((K * ib,), **u8)
        bins = [bin_all[k * bb:(k + 1) * bb] for k in range(K)]
        imgs = [img_all[k * ib:(k + 1) * ib] for k in range(K)]
        with torch.cuda.device(dev):
            _native.check(_lib.gs_forward_bin_views(K, x.P, W0, H0, arr(geoms), nr, arr(bins), arr(imgs),
                                                    int(bool(debug)), _stream(dev), vst), "preprocess_views (binning)")
        out = [(I, radii[k], geoms[k], bounded, bins[k], imgs[k]) for k in range(K)]
    if streams is not None:  # the buffers are used on the views' streams
        for k, s in enumerate(streams):
            for t in out[k][1:]:
                if isinstance(t, torch.Tensor):
                    t.record_stream(s)
    return out


# instance count of the last forward that read it back (bounded forwards do not): a base for a
# binning capacity (last_num_rendered())
_LAST_NUM_RENDERED = [0]


def bounded_status():
    """(flags, instances) that bounded forwards left on the current device since the last call
    (gs_bounded_status; clears them).  Raises RuntimeError when a flag is set."""
    flags, inst = ctypes.c_uint(0), ctypes.c_longlong(0)
    rc = _lib.gs_bounded_status(ctypes.byref(flags), ctypes.byref(inst))
    if rc != 0:
        raise RuntimeError(f"bounded forward: {_native.last_error()}")
    return int(flags.value), int(inst.value)


# forward error flags (include/gsrast.h; gs_internal.h ERR_*): a view with ERR_INVALID set is skipped
# by the backward's record sums and by the fused backward + Adam
ERR_PREFILTERED, ERR_LOOKBACK, ERR_INSTANCES, ERR_CAPACITY = 1, 4, 8, 16
ERR_INVALID = ERR_LOOKBACK | ERR_CAPACITY


def view_flags_word(geom_buffer: torch.Tensor, P: int) -> torch.Tensor:
    """The int32 word of a view's geometry buffer that holds its forward error flags
    (gs_geom_flags_offset, ABI v17), as a one-element device tensor view: copy it out behind the
    forward (non_blocking into pinned memory) to read the view's status at a later sync."""
    off = int(_lib.gs_geom_flags_offset(int(P)))
    if geom_buffer.dtype != torch.uint8 or geom_buffer.numel() < off + 4:
        raise ValueError("view_flags_word: not a geometry buffer of this P")
    return geom_buffer[off:off + 4].view(torch.int32)


class row_waits:
    """Context manager (extension, ABI v17 gs_set_row_waits): the next forward preprocess on this
    thread inside the block launches in Gaussian-row chunks, each behind a stream wait on its
    chunk's event.  waits: [(lo, hi, torch.cuda.Event or None)] covering [0, P) in order.  The
    waits are cleared on exit whether or not a preprocess consumed them."""

    def __init__(self, waits):
        self.waits = list(waits or [])

    def __enter__(self):
        w = self.waits
        if not w:
            return self
        if w[0][0] != 0 or any(w[k][1] != w[k + 1][0] for k in range(len(w) - 1)):
            raise ValueError("row_waits: chunks must be contiguous from row 0")
        bounds = (ctypes.c_int * (len(w) + 1))(*([w[0][0]] + [hi for _, hi, _ in w]))
        evs = (ctypes.c_void_p * len(w))(*[e.cuda_event if e is not None else None for _, _, e in w])
        self._keep = (bounds, evs)
        _native.check(_lib.gs_set_row_waits(len(w), ctypes.cast(bounds, ctypes.c_void_p),
                                            ctypes.cast(evs, ctypes.c_void_p)), "row waits")
        return self

    def __exit__(self, *exc):
        if self.waits:
            _lib.gs_set_row_waits(0, None, None)
        return False


def forward_order_status() -> None:
    """Take the ordering flags of every queued read-back forward on the current device (waits for
    their renders; gs_forward_order_status, ABI v17).  Raises RuntimeError when a look-back wait of
    one of them timed out -- that report is then consumed, not repeated by the next call."""
    if _lib.gs_forward_order_status() != 0:
        raise RuntimeError(_native.last_error())


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, prepared=None, sh_rest=None, capacity=None):
    """prepared: (num_rendered, radii, geomBuffer) of this call from preprocess_views (the first
    half already ran); otherwise both halves run here.  sh_rest: split SH rows (sh is then
    features_dc [P,1,3], sh_rest features_rest [P,M-1,3]; gs_forward_preprocess_split).
    capacity: the binning buffer is sized for that many instances and the whole forward is
    enqueued without a host wait (gs_forward_bounded); the returned num_rendered is the capacity."""
    if _EXT is not None and prepared is not None and capacity is None and sh_rest is None and means3D.is_cuda:
        return _EXT.forward_prepared(background, means3D, viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy),
                                     int(image_height), int(image_width), campos, bool(debug), tuple(prepared))
    if _EXT is not None and prepared is None and capacity is not None and means3D.is_cuda:
        return _EXT.forward_bounded(background, means3D, colors, opacity, scales, rotations, float(scale_modifier),
                                    cov3D_precomp, viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy),
                                    int(image_height), int(image_width), sh, int(degree), campos, bool(prefiltered),
                                    bool(debug), sh_rest, int(capacity))
    if _EXT is not None and prepared is None and capacity is None and means3D.is_cuda:
        out = _EXT.forward(background, means3D, colors, opacity, scales, rotations, float(scale_modifier),
                           cov3D_precomp, viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy), int(image_height),
                           int(image_width), sh, int(degree), campos, bool(prefiltered), bool(debug), sh_rest)
        _LAST_NUM_RENDERED[0] = out[0]
        return out
    x = _Inputs(background, means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh,
                campos, sh_rest=sh_rest)
    if prepared is not None and x.sh_rest is not None:
        raise RuntimeError("split SH rows are not supported with prepared views")
    if prepared is not None and capacity is not None:
        raise RuntimeError("a binning capacity is not supported with prepared views")
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
    if capacity is not None:
        capacity = int(capacity)
        radii = torch.empty((x.P,), dtype=torch.int32, device=dev)
        geom = torch.empty((_lib.gs_geom_buffer_bytes(x.P),), **u8)
        binning = torch.empty((_lib.gs_binning_buffer_bytes(capacity, W, H),), **u8)
        img = torch.empty((_lib.gs_image_buffer_bytes(W, H),), **u8)
        split = x.sh_rest is not None
        with torch.cuda.device(dev):
            _native.check(
                _lib.gs_forward_bounded(
                    x.P, int(degree), x.M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh), _ptr(x.sh_rest),
                    _ptr(x.colors), _ptr(x.opacity), _ptr(x.scales), float(scale_modifier), _ptr(x.rotations),
                    _ptr(x.cov3D), _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy),
                    int(bool(prefiltered)), _ptr(radii), _ptr(geom), capacity, _ptr(binning), _ptr(img),
                    _ptr(out_color), int(bool(debug)), _stream(dev)),
                "rasterize_gaussians (bounded)")
        return capacity, out_color, radii, geom, binning, img
    with torch.cuda.device(dev):
        st = _stream(dev)
        bounded = False
        if prepared is not None:
            num_rendered, radii, geom = prepared[:3]
            bounded = len(prepared) > 3 and prepared[3]
            if radii.numel() != x.P or geom.numel() != _lib.gs_geom_buffer_bytes(x.P):
                raise RuntimeError("rasterize_gaussians: the prepared view does not match these inputs")
            if len(prepared) > 4:  # binned with the other prepared views: the compositing only
                binning, img = prepared[4], prepared[5]
                if img.numel() != _lib.gs_image_buffer_bytes(W, H):
                    raise RuntimeError("rasterize_gaussians: the prepared view was binned for another image size")
                _native.check(
                    _lib.gs_forward_render_binned(
                        x.P, _ptr(x.bg), W, H, _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx),
                        float(tan_fovy), _ptr(geom), num_rendered, _ptr(binning), _ptr(img), _ptr(out_color),
                        int(bool(bounded)), int(bool(debug)), st),
                    "rasterize_gaussians (render)")
                return num_rendered, out_color, radii, geom, binning, img
        else:
            radii = torch.empty((x.P,), dtype=torch.int32, device=dev)
            geom = torch.empty((_lib.gs_geom_buffer_bytes(x.P),), **u8)
            nr = ctypes.c_longlong(0)
            split = x.sh_rest is not None
            _native.check(
                (_lib.gs_forward_preprocess_split if split else _lib.gs_forward_preprocess)(
                    x.P, int(degree), x.M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh),
                    _ptr(x.sh_rest) if split else _ptr(x.colors),
                    _ptr(x.opacity), _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D),
                    _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy),
                    int(bool(prefiltered)), _ptr(radii), _ptr(geom), ctypes.byref(nr), int(bool(debug)), st),
                "rasterize_gaussians (preprocess)")
            num_rendered = int(nr.value)
            _LAST_NUM_RENDERED[0] = num_rendered
        binning = torch.empty((_lib.gs_binning_buffer_bytes(num_rendered, W, H),), **u8)
        img = torch.empty((_lib.gs_image_buffer_bytes(W, H),), **u8)
        _native.check(
            (_lib.gs_forward_render_bounded if bounded else _lib.gs_forward_render)(
                x.P, _ptr(x.bg), W, H, _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy),
                _ptr(radii), _ptr(geom), num_rendered, _ptr(binning), _ptr(img), _ptr(out_color),
                int(bool(debug)), st),
            "rasterize_gaussians (render)")
    return num_rendered, out_color, radii, geom, binning, img


def binning_layout_count(R, binningBuffer, W, H):
    """The instance count binningBuffer is laid out for, which the C-ABI calls take as num_rendered:
    R for a buffer of gs_binning_buffer_bytes(R) bytes (the two-call, bounded and prepared
    forwards); for a buffer the eager forward sized ahead of its count (gs_forward_counted: the
    returned num_rendered is the exact count, the buffer holds the capacity) that capacity."""
    R = int(R)
    n = binningBuffer.numel()
    if n == _lib.gs_binning_buffer_bytes(R, W, H):
        return R
    L = int(_lib.gs_binning_layout_count(n, W, H))
    if L < R:
        raise RuntimeError(f"binningBuffer ({n} bytes) is too small for num_rendered = {R}")
    return L


# gradient outputs of the backward, in the upstream return order, with their GS_ACC_* bit
GRAD_NAMES = ("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations")
GS_ACC = {n: 1 << k for k, n in enumerate(GRAD_NAMES)}


def backward_impl(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                  projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer, R, binningBuffer,
                  imageBuffer, debug, want_all=True, sinks=None, wait_event=None, sh_rest=None):
    """Shared backward.  With want_all=False the gradients that no autograd input can receive
    (colours when SHs drive the colour, cov3D when scale/rotation drive it, ...) are None and
    not computed.  sinks: {name: (buffer, accumulate)} -- that gradient is written into (or, with
    accumulate, added to) the caller's buffer, which is returned in its place
    (gs_backward_accumulate; multi-view gradient buckets, gs_view_parallel.GradBucket).
    wait_event: torch.cuda.Event the stream waits for before the kernel that writes the gradients
    (a sink shared with views on other streams).  sh_rest: split SH rows as rasterize_gaussians;
    the `sh` gradient is then that of the concatenation, [P, M, 3]."""
    if _EXT is not None and not want_all and means3D.is_cuda:
        return _EXT.backward(background, means3D, radii, colors, scales, rotations, float(scale_modifier),
                             cov3D_precomp, viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy), dL_dout_color,
                             sh, int(degree), campos, geomBuffer, int(R), binningBuffer, imageBuffer, bool(debug),
                             sh_rest, sinks or {}, wait_event.cuda_event if wait_event is not None else 0)
    x = _Inputs(background, means3D, colors, None, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh,
                campos, need_opacity=False, sh_rest=sh_rest)
    P, dev = x.P, x.device
    f32 = dict(dtype=torch.float32, device=dev)
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = x.M
    sinks = sinks or {}
    need_col = want_all or x.colors is not None
    need_cov = want_all or x.cov3D is not None
    need_sh = want_all or x.sh is not None
    need_sr = want_all or (x.scales is not None and x.rotations is not None)
    has_sr = x.scales is not None and x.rotations is not None and x.cov3D is None
    shapes = dict(means2D=(P, 3), colors=(P, 3), opacity=(P, 1), means3D=(P, 3), cov3D=(P, 6), sh=(P, M, 3),
                  scales=(P, 3), rotations=(P, 4))
    # is the gradient computed by the kernels (else zero-filled or absent)?
    computed = dict(means2D=True, colors=True, opacity=True, means3D=True,
                    cov3D=x.cov3D is not None or (want_all and has_sr), sh=x.sh is not None, scales=has_sr,
                    rotations=has_sr)
    needed = dict(means2D=True, colors=need_col, opacity=True, means3D=True, cov3D=need_cov, sh=need_sh,
                  scales=need_sr, rotations=need_sr)
    acc = 0
    outs = {}
    for n in GRAD_NAMES:
        if n in sinks and computed[n]:
            buf, accumulate = sinks[n]
            if (buf.dtype != torch.float32 or buf.device != dev or not buf.is_contiguous()
                    or buf.numel() != math.prod(shapes[n])):
                raise RuntimeError(f"gradient sink for {n}: expected a contiguous float32 buffer of "
                                   f"{math.prod(shapes[n])} elements on {dev}")
            outs[n] = buf
            acc |= GS_ACC[n] if accumulate else 0
        elif needed[n]:
            outs[n] = (torch.empty if computed[n] else torch.zeros)(shapes[n], **f32)
        else:
            outs[n] = None
    ret = tuple(outs[n] for n in GRAD_NAMES)
    if P == 0:
        return ret
    dpix = _f32(dL_dout_color, "dL_dout_color", dev)
    o = {n: (outs[n] if computed[n] else None) for n in GRAD_NAMES}
    R = binning_layout_count(R, binningBuffer, W, H)
    with torch.cuda.device(dev):
        st = _stream(dev)
        grad_scratch = torch.empty((_lib.gs_grad_buffer_bytes(R),), dtype=torch.uint8, device=dev)
        wait = ctypes.c_void_p(wait_event.cuda_event) if wait_event is not None else None
        if x.sh_rest is not None:  # split SH rows: SH colours, so no dL/dcolors output
            _native.check(
                _lib.gs_backward_accumulate_split(
                    P, int(degree), M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh), _ptr(x.sh_rest),
                    _ptr(x.opacity), _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D),
                    _ptr(x.view), _ptr(x.proj), _ptr(x.campos), float(tan_fovx), float(tan_fovy), _ptr(radii),
                    _ptr(geomBuffer), int(R), _ptr(binningBuffer), _ptr(imageBuffer), _ptr(dpix), _ptr(grad_scratch),
                    _ptr(o["means2D"]), _ptr(o["opacity"]), _ptr(o["means3D"]), _ptr(o["cov3D"]), _ptr(o["sh"]),
                    _ptr(o["scales"]), _ptr(o["rotations"]), acc, wait, int(bool(debug)), st),
                "rasterize_gaussians_backward")
            return ret
        _native.check(
            _lib.gs_backward_accumulate(
                P, int(degree), M, _ptr(x.bg), W, H, _ptr(x.means3D), _ptr(x.sh), _ptr(x.colors), _ptr(x.opacity),
                _ptr(x.scales), float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D), _ptr(x.view), _ptr(x.proj),
                _ptr(x.campos), float(tan_fovx), float(tan_fovy), _ptr(radii), _ptr(geomBuffer), int(R),
                _ptr(binningBuffer), _ptr(imageBuffer), _ptr(dpix), _ptr(grad_scratch), _ptr(o["means2D"]),
                _ptr(o["colors"]), _ptr(o["opacity"]), _ptr(o["means3D"]), _ptr(o["cov3D"]), _ptr(o["sh"]),
                _ptr(o["scales"]), _ptr(o["rotations"]), acc, wait, int(bool(debug)), st),
            "rasterize_gaussians_backward")
    return ret


def backward_render(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, dL_dout_color, P, degree, M,
                    geomBuffer, R, binningBuffer, imageBuffer, want_means2D, debug):
    """Per-tile half of the backward (gs_backward_render): the view's per-Gaussian record sums,
    kept in geomBuffer for backward_gaussians, and its dL_dmeans2D [P, 3] (or None)."""
    if _EXT is not None and geomBuffer.is_cuda:
        return _EXT.backward_render(background, viewmatrix, projmatrix, campos, float(tan_fovx), float(tan_fovy),
                                    dL_dout_color, int(P), int(degree), int(M), geomBuffer, int(R), binningBuffer,
                                    imageBuffer, bool(want_means2D), bool(debug))
    dev = geomBuffer.device
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    dm2 = torch.empty((P, 3), dtype=torch.float32, device=dev) if want_means2D else None
    if P == 0:
        return dm2
    bg = _f32(background, "background", dev, host_ok=True)
    view = _f32(viewmatrix, "viewmatrix", dev, host_ok=True)
    proj = _f32(projmatrix, "projmatrix", dev, host_ok=True)
    cam = _f32(campos, "campos", dev, host_ok=True)
    dpix = _f32(dL_dout_color, "dL_dout_color", dev)
    R = binning_layout_count(R, binningBuffer, W, H)
    with torch.cuda.device(dev):
        st = _stream(dev)
        grad_scratch = torch.empty((_lib.gs_grad_buffer_bytes(R),), dtype=torch.uint8, device=dev)
        _native.check(
            _lib.gs_backward_render(P, int(degree), int(M), _ptr(bg), W, H, _ptr(view), _ptr(proj), _ptr(cam),
                                    float(tan_fovx), float(tan_fovy), _ptr(geomBuffer), int(R), _ptr(binningBuffer),
                                    _ptr(imageBuffer), _ptr(dpix), _ptr(grad_scratch), _ptr(dm2), 0,
                                    int(bool(debug)), st),
            "rasterize_gaussians_backward (render half)")
    return dm2


def backward_gaussians(means3D, sh, colors, scales, rotations, cov3D_precomp, scale_modifier, degree, views, outs,
                       accumulate, wait_event=None, debug=False, first=0, count=None):
    """Per-Gaussian half of the backward for several views at once (gs_backward_gaussians).
    views: [(viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, W, H, geomBuffer)] in order (each
    after its backward_render); outs: {name: buffer} for colors / opacity / means3D / cov3D / sh /
    scales / rotations (absent: not produced); accumulate: GS_ACC bits of the first view.
    first / count: only the Gaussians [first, first + count) (gs_backward_gaussians_range)."""
    if _EXT is not None and means3D.is_cuda:
        return _EXT.backward_gaussians(means3D, sh, colors, scales, rotations, cov3D_precomp, float(scale_modifier),
                                       int(degree), views, outs, int(accumulate),
                                       wait_event.cuda_event if wait_event is not None else 0, bool(debug),
                                       int(first), -1 if count is None else int(count))
    x = _Inputs(None, means3D, colors, None, scales, rotations, cov3D_precomp, views[0][0],
                views[0][1], sh, views[0][2], need_opacity=False)
    P, dev = x.P, x.device
    if P == 0 or not views:
        return
    arr = (_native.ViewGrad * len(views))()
    keep = []
    for k, (vm, pm, cp, tx, ty, W, H, geom) in enumerate(views):
        vm, pm = _f32(vm, "viewmatrix", dev, host_ok=True), _f32(pm, "projmatrix", dev, host_ok=True)
        cp = _f32(cp, "campos", dev, host_ok=True)
        keep += [vm, pm, cp]
        arr[k] = _native.ViewGrad(vm.data_ptr(), pm.data_ptr(), cp.data_ptr() if cp is not None else None,
                                  float(tx), float(ty), int(W), int(H), geom.data_ptr())
    o = {n: outs.get(n) for n in ("colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations")}
    for n, t in o.items():
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev):
            raise RuntimeError(f"backward_gaussians: {n} output must be a contiguous float32 tensor on {dev}")
    count = P - int(first) if count is None else int(count)
    with torch.cuda.device(dev):
        _native.check(
            _lib.gs_backward_gaussians_range(
                P, int(first), count, int(degree), x.M, _ptr(x.means3D), _ptr(x.sh), _ptr(x.colors), _ptr(x.scales),
                float(scale_modifier), _ptr(x.rotations), _ptr(x.cov3D), len(views), arr, _ptr(o["colors"]),
                _ptr(o["opacity"]), _ptr(o["means3D"]), _ptr(o["cov3D"]), _ptr(o["sh"]), _ptr(o["scales"]),
                _ptr(o["rotations"]), int(accumulate),
                ctypes.c_void_p(wait_event.cuda_event) if wait_event is not None else None, int(bool(debug)),
                _stream(dev)),
            "rasterize_gaussians_backward (per-Gaussian half)")


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
    v = _f32(viewmatrix, "viewmatrix", dev, host_ok=True)
    p = _f32(projmatrix, "projmatrix", dev, host_ok=True)
    with torch.cuda.device(dev):
        _native.check(_lib.gs_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(dev)), "mark_visible")
    return present


def debug_export(P, W, H, num_rendered, geomBuffer, binningBuffer, imageBuffer, device):
    """Forward intermediates for tests: dict of device tensors."""
    u32 = dict(dtype=torch.int32, device=device)
    f32 = dict(dtype=torch.float32, device=device)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    L = binning_layout_count(num_rendered, binningBuffer, W, H) if P > 0 else int(num_rendered)
    out = dict(
        point_list=torch.zeros((max(L, 1),), **u32),
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
                _lib.gs_debug_export(P, W, H, L, _ptr(geomBuffer), _ptr(binningBuffer),
                                     _ptr(imageBuffer), *[_ptr(out[k]) for k in (
                                         "point_list", "ranges", "xy", "conic_opacity", "rgb", "depth",
                                         "tiles_touched", "final_T", "n_contrib")], _stream(device)),
                "debug_export")
    out["point_list"] = out["point_list"][:num_rendered]
    return out


def debug_export_slots(W, H, num_rendered, binningBuffer, imageBuffer, device):
    """(slots[num_rendered], tile_cut[tiles]) as int32 device tensors: the depth-ordered instance slot of
    each entry of the tile-sorted list and each tile's backward record cut (valid after a backward)."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    L = binning_layout_count(num_rendered, binningBuffer, W, H)
    slots = torch.zeros((max(L, 1),), dtype=torch.int32, device=device)
    cuts = torch.zeros((gx * gy,), dtype=torch.int32, device=device)
    with torch.cuda.device(device):
        _native.check(_lib.gs_debug_export_slots(W, H, L, _ptr(binningBuffer), _ptr(imageBuffer),
                                                 _ptr(slots), _ptr(cuts), _stream(device)), "debug_export_slots")
    return slots[:int(num_rendered)], cuts
