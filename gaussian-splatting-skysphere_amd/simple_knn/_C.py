"""`simple_knn._C.distCUDA2(points[P, 3]) -> float[P]`: mean squared distance of each point to its
3 nearest other points, computed by libgsrast.so (gs_knn_mean_dist2, hand-written HIP for gfx950).
Same name and meaning as the un-vendored upstream extension (/root/reference/.gitmodules:1-3)."""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _native

_lib = _native.load()


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if points.ndimension() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    if not points.is_cuda:
        raise RuntimeError("distCUDA2 (MI355X/HIP) needs a device tensor; there is no CPU path")
    pts = points.float().contiguous()
    P = pts.size(0)
    out = torch.empty((P,), dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    with torch.cuda.device(pts.device):
        scratch = torch.empty((_lib.gs_knn_scratch_bytes(P),), dtype=torch.uint8, device=pts.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(pts.device).cuda_stream)
        _native.check(_lib.gs_knn_mean_dist2(P, ctypes.c_void_p(pts.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                             ctypes.c_void_p(scratch.data_ptr()), st), "distCUDA2")
    return out
