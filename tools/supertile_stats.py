"""Binning-granularity study for DESIGN §10 (coarser binning): the C3 scene through the CPU oracle
binned at 16x16 tiles (the build) and at 32x32 super-tiles (an oracle build with TILE = 32, path
in argv[1]; made by tools/supertile_stats.sh).  Prints the instance counts (what the duplicate, the
tile sort, the ranges and the record sums scale with) and the entries the render kernels would
stage per wave when every 16x16 tile (backward workgroup) or 8x8 quadrant (forward wave) walks its
super-tile's list instead of its own.  The composited images of the two builds are compared too
(binning changes no pixel).  Analysis only: nothing here is on the product path."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import gs_scenes  # noqa: E402
from oracle import gs_oracle  # noqa: E402

P, DEG, W, H = int(os.environ.get("ST_P", 1_000_000)), 3, 1920, 1080


def run(lib_path, tile):
    gs_oracle._LIB_PATH = lib_path
    gs_oracle._lib = None
    gs_oracle.set_threads(os.cpu_count() or 8)
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(P, DEG, cam=cam, seed=0)
    osc = gs_oracle.Scene(bg=np.zeros(3, np.float32), means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(),
                          W=W, H=H, viewmatrix=cam.world_view_transform.numpy(),
                          projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                          tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2), shs=sc.shs.numpy(),
                          sh_degree=DEG, scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
    out = gs_oracle.forward(osc, intermediates=True)
    gx, gy = (W + tile - 1) // tile, (H + tile - 1) // tile
    rng = out["ranges"][: gx * gy].astype(np.int64)
    n_list = (rng[:, 1] - rng[:, 0]).reshape(gy, gx)
    return out, n_list


def block_max(a, b):
    """max of a [H, W] array over b x b blocks (padded with 0)"""
    hh, ww = -(-a.shape[0] // b) * b, -(-a.shape[1] // b) * b
    p = np.zeros((hh, ww), a.dtype)
    p[: a.shape[0], : a.shape[1]] = a
    return p.reshape(hh // b, b, ww // b, b).max(axis=(1, 3))


def staged(walk, n):
    """entries staged in 64-entry batches until the walk's last entry (at most the list)"""
    return np.minimum(n, -(-walk // 64) * 64)


def diff_report(o16, o32):
    """pixels whose composite differs between the two binnings, and the largest difference"""
    d = np.abs(o16["color"] - o32["color"]).max(axis=0)
    dt = np.abs(o16["final_T"] - o32["final_T"])
    return {"pixels_color_differ": int((d > 0).sum()), "max_color_diff": float(d.max()),
            "pixels_T_differ": int((dt > 0).sum()), "max_T_diff": float(dt.max())}


def main():
    lib16 = os.path.join(ROOT, "oracle", "build", "libgs_oracle.so")
    lib32 = sys.argv[1]
    o16, n16 = run(lib16, 16)
    o32, n32 = run(lib32, 32)
    same = np.array_equal(o16["color"], o32["color"]) and np.array_equal(o16["final_T"], o32["final_T"])
    nc16, nc32 = o16["n_contrib"].astype(np.int64), o32["n_contrib"].astype(np.int64)
    # backward: each 16x16 tile walks its list up to its largest n_contrib
    w16 = np.minimum(block_max(nc16, 16), n16)
    n32_per16 = np.repeat(np.repeat(n32, 2, axis=0), 2, axis=1)[: n16.shape[0], : n16.shape[1]]
    w32 = np.minimum(block_max(nc32, 16), n32_per16)
    # forward: each 8x8 quadrant wave stages its tile's (super-tile's) list until its pixels stop
    q16 = block_max(nc16, 8)
    q32 = block_max(nc32, 8)
    nq16 = np.repeat(np.repeat(n16, 2, axis=0), 2, axis=1)[: q16.shape[0], : q16.shape[1]]
    nq32 = np.repeat(np.repeat(n32, 4, axis=0), 4, axis=1)[: q32.shape[0], : q32.shape[1]]
    res = {
        "P": P, "images_identical": bool(same),
        "instances_16": int(o16["num_rendered"]), "instances_32": int(o32["num_rendered"]),
        "bwd_walk_entries_16": int(w16.sum()), "bwd_walk_entries_32": int(w32.sum()),
        "bwd_staged_16": int(staged(w16, n16).sum()), "bwd_staged_32": int(staged(w32, n32_per16).sum()),
        "fwd_staged_16": int(staged(q16, nq16).sum()), "fwd_staged_32": int(staged(q32, nq32).sum()),
        "records_walked_32_per_subtile": int(w32.sum()),
    }
    res.update(diff_report(o16, o32))
    for k, v in res.items():
        print(f"{k:32s} {v}")


if __name__ == "__main__":
    main()
