"""Backward-walk layout study: how many (entry, pixel-rectangle) evaluations a
render-backward layout would issue on the C3 scene, computed from the CPU oracle's forward
(point lists, n_contrib, splat records).  For every tile entry a tile walk reaches (slot <
the tile's largest n_contrib) it counts, per candidate sub-rectangle of the tile (two 8x16 column
halves = the round-3 kernel's waves; four 8x8 quadrants; four 16x4 row bands), whether the
entry's alpha >= 1/255 ellipse meets the rectangle (the cull the kernel applies), whether the
rectangle's walk still reaches the entry (slot < its largest n_contrib) and whether any pixel of it
actually contributes.  Analysis only: nothing here is on the product path."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import gs_scenes  # noqa: E402
from oracle import gs_oracle  # noqa: E402

P = int(os.environ.get("ST_P", 1_000_000))
W, H, DEG = int(os.environ.get("ST_W", 1920)), int(os.environ.get("ST_H", 1080)), 3


def rect_meets(mx, my, cx, cy, cz, lim, x0, x1, y0, y1):
    """numpy restatement of ellipse_meets_rect (gs_common.h): conservative alpha >= 1/255 test"""
    dxl, dxh, dyl, dyh = x0 - mx, x1 - mx, y0 - my, y1 - my
    inside = (dxl <= 0) & (dxh >= 0) & (dyl <= 0) & (dyh >= 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        icx, icz = 1.0 / cx, 1.0 / cz

        def q(dx, dy):
            return cx * dx * dx + 2 * cy * dx * dy + cz * dy * dy

        b = q(dxl, np.clip(-cy * dxl * icz, dyl, dyh))
        b = np.minimum(b, q(dxh, np.clip(-cy * dxh * icz, dyl, dyh)))
        b = np.minimum(b, q(np.clip(-cy * dyl * icx, dxl, dxh), dyl))
        b = np.minimum(b, q(np.clip(-cy * dyh * icx, dxl, dxh), dyh))
    return (lim >= 0) & (inside | ~((cx > 0) & (cz > 0)) | (b <= lim))


def main():
    gs_oracle.set_threads(os.cpu_count() or 8)
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(P, DEG, cam=cam, seed=0)
    osc = gs_oracle.Scene(bg=np.zeros(3, np.float32), means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(),
                          W=W, H=H, viewmatrix=cam.world_view_transform.numpy(),
                          projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                          tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2), shs=sc.shs.numpy(),
                          sh_degree=DEG, scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
    out = gs_oracle.forward(osc, intermediates=True)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    nc = np.zeros((gy * 16, gx * 16), np.int64)
    nc[:H, :W] = out["n_contrib"]
    # per tile [16, 16] n_contrib
    ncT = nc.reshape(gy, 16, gx, 16).transpose(0, 2, 1, 3).reshape(gy * gx, 16, 16)
    rng = out["ranges"][: gx * gy].astype(np.int64)
    nlist = rng[:, 1] - rng[:, 0]
    n_eff = np.minimum(ncT.reshape(-1, 256).max(1), nlist)
    lst = out["point_list"].astype(np.int64)
    xy, co = out["xy"], out["conic_opacity"]
    o = co[:, 3].astype(np.float64)
    with np.errstate(divide="ignore"):
        lim_all = np.where(o >= 1 / 255, 2 * np.log(255 * o) * 1.001 + 1e-3, -1.0)
    # rectangles: (name, list of (x0, x1, y0, y1) in tile-local pixel coords, pixel masks [16,16])
    yy, xx = np.mgrid[0:16, 0:16]
    layouts = {
        "half": [(0, 7, 0, 15), (8, 15, 0, 15)],
        "quad": [(0, 7, 0, 7), (8, 15, 0, 7), (0, 7, 8, 15), (8, 15, 8, 15)],
        "band4": [(0, 15, 4 * k, 4 * k + 3) for k in range(4)],
        "tile": [(0, 15, 0, 15)],
    }
    stats = {k: dict(meets=0, reach=0, contrib=0) for k in layouts}
    tiles = np.nonzero(n_eff > 0)[0]
    total_entries = int(n_eff.sum())
    contrib_pairs = 0
    pix_x = xx.reshape(-1).astype(np.float32)
    pix_y = yy.reshape(-1).astype(np.float32)
    CH = 4000
    for c0 in range(0, len(tiles), CH):
        tb = tiles[c0:c0 + CH]
        cnt = n_eff[tb]
        t_rep = np.repeat(tb, cnt)
        e = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        gid = lst[rng[t_rep, 0] + e]
        ox = (t_rep % gx) * 16.0
        oy = (t_rep // gx) * 16.0
        mx = xy[gid, 0] - ox
        my = xy[gid, 1] - oy
        cx, cy, cz, op = co[gid, 0], co[gid, 1], co[gid, 2], co[gid, 3]
        lim = lim_all[gid]
        # per pixel contribution (float32 like the kernels; exact decisions do not matter here)
        dx = mx[:, None] - pix_x[None, :]
        dy = my[:, None] - pix_y[None, :]
        power = -0.5 * (cx[:, None] * dx * dx + cz[:, None] * dy * dy) - cy[:, None] * dx * dy
        alpha = np.minimum(0.99, op[:, None] * np.exp(power))
        live = e[:, None] < ncT[t_rep].reshape(-1, 256)
        con = (alpha >= 1 / 255) & (power <= 0) & live
        contrib_pairs += int(con.sum())
        con = con.reshape(-1, 16, 16)
        ncb = ncT[t_rep]
        for name, rects in layouts.items():
            s = stats[name]
            for (x0, x1, y0, y1) in rects:
                m = rect_meets(mx, my, cx, cy, cz, lim, float(x0), float(x1), float(y0), float(y1))
                last = ncb[:, y0:y1 + 1, x0:x1 + 1].reshape(len(e), -1).max(1)
                r = m & (e < last)
                s["meets"] += int(m.sum())
                s["reach"] += int(r.sum())
                s["contrib"] += int((r & con[:, y0:y1 + 1, x0:x1 + 1].reshape(len(e), -1).any(1)).sum())
    print(f"P {P}  {W}x{H}  instances {out['num_rendered']}  walked entries {total_entries}")
    print(f"contributing (pixel, entry) pairs {contrib_pairs}  per walked entry {contrib_pairs / total_entries:.1f}")
    for name, s in stats.items():
        n = len(layouts[name])
        print(f"{name:6s} rects {n}: meets {s['meets']:>10d}  evaluated (reached) {s['reach']:>10d} "
              f"({s['reach'] / total_entries:.3f} per entry)  with a contributor {s['contrib']:>10d} "
              f"({s['contrib'] / total_entries:.3f} per entry)  pixel slots evaluated per entry "
              f"{s['reach'] / total_entries * 256 / n:.1f}")


if __name__ == "__main__":
    main()
