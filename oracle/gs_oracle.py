"""ctypes front-end of the CPU oracle (oracle/gs_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  It
restates the reference rasterizer's algorithm (call site
/root/reference/gaussian_renderer/__init__.py:85-93) on the CPU; the product package never
imports it.

All arrays are numpy float32 / int32 / uint32, C-contiguous, on the host.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libgs_oracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)
_u = ctypes.POINTER(ctypes.c_uint32)
_b = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "gs_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_exp.restype = ctypes.c_float
        L.oracle_exp.argtypes = [ctypes.c_float]
        L.oracle_log.restype = ctypes.c_float
        L.oracle_log.argtypes = [ctypes.c_float]
        L.oracle_set_near_flags.argtypes = [ctypes.c_void_p]
        L.oracle_forward.restype = ctypes.c_longlong
        L.oracle_backward.restype = ctypes.c_longlong
        _lib = L
    return _lib


def _p(a, t=_f):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(t)


def _f32(a):
    if a is None:
        return None
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return a if a.size > 0 else None


class Scene:
    """Inputs of one rasterizer call (host copies, fp32)."""

    def __init__(self, bg, means3D, opacities, W, H, viewmatrix, projmatrix, campos, tanfovx, tanfovy,
                 shs=None, sh_degree=0, colors_precomp=None, scales=None, rotations=None,
                 cov3D_precomp=None, scale_modifier=1.0):
        self.bg = _f32(bg)
        self.means3D = _f32(means3D).reshape(-1, 3) if _f32(means3D) is not None else np.zeros((0, 3), np.float32)
        self.P = self.means3D.shape[0]
        self.opacities = _f32(opacities)
        self.W, self.H = int(W), int(H)
        self.view = _f32(viewmatrix)
        self.proj = _f32(projmatrix)
        self.campos = _f32(campos)
        self.tanfovx, self.tanfovy = float(tanfovx), float(tanfovy)
        self.shs = _f32(shs)
        self.M = 0 if self.shs is None else self.shs.reshape(self.P, -1, 3).shape[1]
        self.D = int(sh_degree)
        self.colors = _f32(colors_precomp)
        self.scales = _f32(scales)
        self.rots = _f32(rotations)
        self.cov3D = _f32(cov3D_precomp)
        self.mod = float(scale_modifier)

    def _common(self):
        return (self.P, self.D, self.M, _p(self.bg), self.W, self.H, _p(self.means3D), _p(self.shs),
                _p(self.colors), _p(self.opacities), _p(self.scales), ctypes.c_float(self.mod),
                _p(self.rots), _p(self.cov3D), _p(self.view), _p(self.proj), _p(self.campos),
                ctypes.c_float(self.tanfovx), ctypes.c_float(self.tanfovy))


def forward(sc: Scene, intermediates: bool = False, near: bool = False):
    """Returns dict(color[3,H,W], radii[P], num_rendered, and intermediates if asked).
    near=True adds near[H,W] (uint8): pixels with a decision close to the alpha / T thresholds
    (see oracle_set_near_flags in gs_oracle.c), for comparisons with the device's fast exp2."""
    L = lib()
    if near:
        flags = np.zeros((sc.H, sc.W), np.uint8)
        L.oracle_set_near_flags(flags.ctypes.data_as(ctypes.c_void_p))
        try:
            out = forward(sc, intermediates)
        finally:
            L.oracle_set_near_flags(None)
        out["near"] = flags
        return out
    P, W, H = sc.P, sc.W, sc.H
    gx, gy = (W + 15) // 16, (H + 15) // 16
    color = np.zeros((3, H, W), np.float32)
    radii = np.zeros((P,), np.int32)
    out = dict(color=color, radii=radii)
    xy = np.zeros((P, 2), np.float32)
    co = np.zeros((P, 4), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    depth = np.zeros((P,), np.float32)
    tiles = np.zeros((P,), np.uint32)
    clamped = np.zeros((P, 3), np.uint8)
    finalT = np.zeros((H, W), np.float32)
    ncon = np.zeros((H, W), np.uint32)
    ranges = np.zeros((gx * gy, 2), np.uint32)
    args = sc._common() + (_p(color), _p(radii, _i))
    if intermediates:
        I = L.oracle_forward(*args, _p(xy), _p(co), _p(rgb), _p(depth), _p(tiles, _u), _p(clamped, _b),
                             _p(finalT), _p(ncon, _u), None, _p(ranges, _u))
        lst = np.zeros((max(I, 1),), np.uint32)
        L.oracle_forward(*args, None, None, None, None, None, None, None, None, _p(lst, _u), None)
        out.update(xy=xy, conic_opacity=co, rgb=rgb, depth=depth, tiles_touched=tiles, clamped=clamped,
                   final_T=finalT, n_contrib=ncon, ranges=ranges, point_list=lst[:I])
    else:
        I = L.oracle_forward(*args, None, None, None, None, None, None, None, None, None, None)
    out["num_rendered"] = int(I)
    return out


def backward(sc: Scene, dL_dpix):
    """Returns the 8 upstream gradients (+ dconic), each [P, ...] float32."""
    L = lib()
    P = sc.P
    M = max(sc.M, 1)
    g = dict(
        dmeans2D=np.zeros((P, 3), np.float32),
        dcolors=np.zeros((P, 3), np.float32),
        dopacity=np.zeros((P, 1), np.float32),
        dmeans3D=np.zeros((P, 3), np.float32),
        dcov3D=np.zeros((P, 6), np.float32),
        dsh=np.zeros((P, M, 3), np.float32),
        dscales=np.zeros((P, 3), np.float32),
        drotations=np.zeros((P, 4), np.float32),
        dconic=np.zeros((P, 2, 2), np.float32),
    )
    dpix = _f32(dL_dpix)
    I = L.oracle_backward(*sc._common(), _p(dpix), _p(g["dmeans2D"]), _p(g["dcolors"]), _p(g["dopacity"]),
                          _p(g["dmeans3D"]), _p(g["dcov3D"]), _p(g["dsh"]), _p(g["dscales"]),
                          _p(g["drotations"]), _p(g["dconic"]))
    g["num_rendered"] = int(I)
    return g


def set_threads(n: int):
    """OpenMP threads for render / preprocess loops (results do not depend on it)."""
    lib().oracle_set_threads(int(n))


def exp(x: float) -> float:
    return float(lib().oracle_exp(ctypes.c_float(x)))


def log(x: float) -> float:
    return float(lib().oracle_log(ctypes.c_float(x)))


def set_exact_tiles(on: bool):
    """Tile-exact binning (default, = the HIP path) or the full upstream tile rectangle."""
    lib().oracle_set_exact_tiles(int(bool(on)))


def set_acc_f32(on: bool):
    """Backward sums in fp32 (this oracle's order) instead of fp64: the fp32 ordering-noise probe
    the conditioning-aware gradient checks compare the device against (gs_oracle.c)."""
    lib().oracle_set_acc_f32(int(bool(on)))


def backward_f32_acc(sc: Scene, dL_dpix):
    """backward() with fp32 accumulation (set_acc_f32), restoring the fp64 default afterwards."""
    set_acc_f32(True)
    try:
        return backward(sc, dL_dpix)
    finally:
        set_acc_f32(False)


def sh_forward(deg, means, campos, shs):
    P = means.shape[0]
    shs = _f32(shs).reshape(P, -1, 3)
    M = shs.shape[1]
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    lib().oracle_sh_forward(P, deg, M, _p(_f32(means)), _p(_f32(campos)), _p(shs), _p(rgb), _p(clamped, _b))
    return rgb, clamped


def sh_backward(deg, means, campos, shs, clamped, drgb):
    P = means.shape[0]
    shs = _f32(shs).reshape(P, -1, 3)
    M = shs.shape[1]
    dsh = np.zeros((P, M, 3), np.float32)
    dmean = np.zeros((P, 3), np.float32)
    lib().oracle_sh_backward(P, deg, M, _p(_f32(means)), _p(_f32(campos)), _p(shs),
                             _p(np.ascontiguousarray(clamped, np.uint8), _b), _p(_f32(drgb)), _p(dsh), _p(dmean))
    return dsh, dmean


def cov3d(scales, mod, rots):
    P = scales.shape[0]
    cov = np.zeros((P, 6), np.float32)
    lib().oracle_cov3d(P, _p(_f32(scales)), ctypes.c_float(mod), _p(_f32(rots)), _p(cov))
    return cov


def cov3d_backward(scales, mod, rots, dcov):
    P = scales.shape[0]
    ds = np.zeros((P, 3), np.float32)
    dr = np.zeros((P, 4), np.float32)
    lib().oracle_cov3d_backward(P, _p(_f32(scales)), ctypes.c_float(mod), _p(_f32(rots)), _p(_f32(dcov)),
                                _p(ds), _p(dr))
    return ds, dr


def mark_visible(means, view, proj):
    P = means.shape[0]
    out = np.zeros((P,), np.uint8)
    lib().oracle_mark_visible(P, _p(_f32(means)), _p(_f32(view)), _p(_f32(proj)), _p(out, _b))
    return out.astype(bool)


def knn_mean_dist2(points):
    pts = _f32(points).reshape(-1, 3)
    out = np.zeros((pts.shape[0],), np.float32)
    lib().oracle_knn_mean_dist2(pts.shape[0], _p(pts), _p(out))
    return out
