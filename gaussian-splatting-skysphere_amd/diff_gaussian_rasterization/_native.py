"""Loader for libgsrast.so, the MI355X (gfx950) HIP rasterizer behind include/gsrast.h.

There is no fallback: if the shared library is missing or does not load, importing
`diff_gaussian_rasterization._C` raises.  Build it with `make -C gaussian-splatting-skysphere_amd`
(or `python __graft_entry__.py build`).
"""
from __future__ import annotations

import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GSRAST_LIB", os.path.join(_PKG_ROOT, "build", "libgsrast.so"))

_c_p = ctypes.c_void_p
_c_i = ctypes.c_int
_c_d = ctypes.c_double
_c_f = ctypes.c_float
_c_ll = ctypes.c_longlong
_c_sz = ctypes.c_size_t



class ViewGrad(ctypes.Structure):
    """gs_view_grad (include/gsrast.h): one view of a multi-view per-Gaussian backward."""
    _fields_ = [("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p), ("campos", ctypes.c_void_p),
                ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float), ("image_width", ctypes.c_int),
                ("image_height", ctypes.c_int), ("geom_buffer", ctypes.c_void_p)]


# name -> (restype, argtypes); mirrors include/gsrast.h
SIGNATURES = {
    "gs_abi_version": (_c_i, []),
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_geom_buffer_bytes": (_c_sz, [_c_i]),
    "gs_binning_buffer_bytes": (_c_sz, [_c_ll, _c_i, _c_i]),
    "gs_image_buffer_bytes": (_c_sz, [_c_i, _c_i]),
    "gs_grad_buffer_bytes": (_c_sz, [_c_ll]),
    "gs_forward_preprocess": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_i, _c_p, _c_p, ctypes.POINTER(_c_ll), _c_i, _c_p],
    ),
    "gs_forward_preprocess_views": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_p, _c_p, _c_i, _c_p, _c_p, ctypes.POINTER(_c_ll), _c_i, _c_p, _c_p],
    ),
    "gs_forward_render": (
        _c_i,
        [_c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_f, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_i, _c_p],
    ),
    "gs_rasterize_forward": (
        _c_ll,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_p],
    ),
    "gs_backward": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_i, _c_p],
    ),
    "gs_backward_accumulate": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
         ctypes.c_uint, _c_p, _c_i, _c_p],
    ),
    # ABI v8: features_dc / features_rest in place of shs (and of colors_precomp / dL_dcolors)
    "gs_forward_preprocess_split": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_i, _c_p, _c_p, ctypes.POINTER(_c_ll), _c_i, _c_p],
    ),
    "gs_backward_accumulate_split": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
         ctypes.c_uint, _c_p, _c_i, _c_p],
    ),
    "gs_backward_render": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_f, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_p,
         _c_p, ctypes.c_uint, _c_i, _c_p],
    ),
    "gs_backward_gaussians": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_i, ctypes.POINTER(ViewGrad), _c_p, _c_p,
         _c_p, _c_p, _c_p, _c_p, _c_p, ctypes.c_uint, _c_p, _c_i, _c_p],
    ),
    # ABI v9: the per-Gaussian half for the Gaussians [first, first + count)
    "gs_backward_gaussians_range": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_i, ctypes.POINTER(ViewGrad), _c_p,
         _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, ctypes.c_uint, _c_p, _c_i, _c_p],
    ),
    # ABI v10: the whole forward without a host wait (binning buffer sized ahead) and its sticky status
    "gs_forward_bounded": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_i, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_i, _c_p],
    ),
    "gs_bounded_status": (_c_i, [ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(_c_ll)]),
    "gs_forward_preprocess_views_bounded": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_p, _c_p, _c_i, _c_p, _c_p, ctypes.POINTER(_c_ll), _c_i, _c_p, _c_p],
    ),
    "gs_forward_render_bounded": (
        _c_i,
        [_c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_f, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_i, _c_p],
    ),
    # ABI v11: the binning of K prepared views in one set of launches, then each view's compositing
    "gs_forward_bin_views": (_c_i, [_c_i, _c_i, _c_i, _c_i, _c_p, ctypes.POINTER(_c_ll), _c_p, _c_p, _c_i, _c_p, _c_p]),
    "gs_forward_render_binned": (
        _c_i,
        [_c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_f, _c_p, _c_ll, _c_p, _c_p, _c_p, _c_i, _c_i, _c_p],
    ),
    # ABI v14: the eager forward with its instance count read back at the end
    "gs_forward_counted": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_f, _c_f, _c_i, _c_p, _c_p, _c_ll, _c_p, _c_p, _c_p, ctypes.POINTER(_c_ll), _c_i, _c_p],
    ),
    "gs_binning_layout_count": (_c_ll, [_c_sz, _c_i, _c_i]),
    # ABI v15: one view's per-Gaussian backward half fused with the six groups' Adam step
    "gs_backward_gaussians_adam": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, ctypes.POINTER(ViewGrad), _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_p, _c_d, _c_d, _c_d, _c_i, _c_i, _c_p],
    ),
    # ABI v16: the same plus the view's densification statistics in that pass
    "gs_backward_gaussians_adam_stats": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, ctypes.POINTER(ViewGrad), _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_p, _c_d, _c_d, _c_d, _c_i, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_i, _c_p],
    ),
    # ABI v17: a view's forward error-flags word (its offset in the geometry buffer) and the
    # read-back forwards' ordering status, taken in the caller's own call
    "gs_geom_flags_offset": (_c_sz, [_c_i]),
    "gs_forward_order_status": (_c_i, []),
    "gs_set_row_waits": (_c_i, [_c_i, _c_p, _c_p]),
    "gs_mark_visible": (_c_i, [_c_i, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "gs_knn_scratch_bytes": (_c_sz, [_c_i]),
    "gs_knn_mean_dist2": (_c_i, [_c_i, _c_p, _c_p, _c_p, _c_p]),
    "gs_set_exact_exp": (_c_i, [_c_i]),
    "gs_debug_launch_log": (_c_i, [_c_i]),
    "gs_debug_launched_kernels": (_c_ll, [ctypes.c_char_p, _c_ll]),
    "gs_ssim_partial_count": (_c_sz, [_c_i, _c_i, _c_i]),
    "gs_ssim_forward": (_c_i, [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "gs_ssim_backward": (_c_i, [_c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "gs_photometric_loss_forward": (_c_i, [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p]),
    "gs_photometric_loss_backward": (_c_i, [_c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p]),
    "gs_adam_step": (_c_i, [_c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_d, _c_d, _c_d, _c_i, _c_p]),
    "gs_adam_step_activated": (_c_i, [_c_i, _c_p, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_d, _c_d, _c_d,
                                      _c_i, _c_p]),
    "gs_activate_forward": (_c_i, [_c_i, _c_i] + [_c_p] * 9 + [_c_p]),
    "gs_activate_backward": (_c_i, [_c_i, _c_i] + [_c_p] * 12 + [_c_p]),
    "gs_densify_block_count": (_c_sz, [_c_i]),
    "gs_densify_classify": (_c_i, [_c_i, _c_p, _c_p, _c_p, _c_p, _c_d, _c_d, _c_d, _c_d, _c_i, _c_d, _c_i, _c_p, _c_p,
                                   _c_p, _c_p]),
    "gs_densify_split_stds": (_c_i, [_c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "gs_densify_emit": (_c_i, [_c_i, _c_i] + [_c_p] * 12),
    "gs_densify_stats": (_c_i, [_c_i, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_p]),
    "gs_debug_export": (
        _c_i,
        [_c_i, _c_i, _c_i, _c_ll, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    ),
    "gs_debug_export_slots": (_c_i, [_c_i, _c_i, _c_ll, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "gs_debug_set_scan_spin_limit": (ctypes.c_uint, [ctypes.c_uint]),
    "gs_profile_enable": (None, [_c_i]),
    "gs_profile_collect": (_c_i, []),
    "gs_profile_reset": (None, []),
    "gs_profile_stat": (_c_i, [_c_i, ctypes.c_char_p, _c_i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_ll)]),
}

_lib = None


def load():
    """Load libgsrast.so once and declare every C-ABI symbol.  Raises if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgsrast.so not found at {LIB_PATH}; build it with "
            f"`make -C {_PKG_ROOT}` (hipcc --offload-arch=gfx950). There is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().gs_last_error()
    return msg.decode() if msg else "unknown error"


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what}: {last_error()}")


def profile_stats():
    """Per-kernel (name -> (total_ms, launches)) collected with gs_profile_enable(1)."""
    lib = load()
    lib.gs_profile_collect()
    out = {}
    i = 0
    buf = ctypes.create_string_buffer(128)
    ms = ctypes.c_double()
    n = ctypes.c_longlong()
    while lib.gs_profile_stat(i, buf, 128, ctypes.byref(ms), ctypes.byref(n)):
        out[buf.value.decode()] = (ms.value, n.value)
        i += 1
    return out
