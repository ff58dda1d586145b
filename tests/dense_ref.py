"""Dense, differentiable PyTorch restatement of the rasterizer (test infrastructure).

Independent of oracle/gs_oracle.c: written directly from the spec with
torch autograd providing the backward, so it checks the oracle's hand-derived gradients.  Small
scenes only (loops over Gaussians, vectorised over pixels).  Deliberate mirrors of upstream
behaviour that autograd would not produce on its own:
  - alpha = min(0.99, o*G) with the clamp NOT gating the gradient (straight-through);
  - the quaternion is used un-normalised;
  - past the 1.3x FoV clamp of the EWA Jacobian the clamped t.x / t.y is held constant (upstream
    zeroes dL/dt.x there and differentiates J through t.z with the clamped t.x fixed);
  - per-pixel candidate sets are the tile rectangles of the 3-sigma radius (tile binning).
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def sh_rgb(deg, sh, d):
    """sh [P, K, 3], d [P, 3] unit -> [P, 3] before +0.5 / clamp."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r


def quat_R(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1),
    ], -2)


def _prep(means3D, means2D, opac, view, proj, campos, tanfovx, tanfovy, W, H, shs=None, deg=0, colors=None,
          scales=None, rots=None, cov3D=None, mod=1.0):
    """The per-Gaussian half (projection, EWA covariance, conic, radius, colour, tile rectangle)."""
    dt = means3D.dtype
    P = means3D.shape[0]
    ones = torch.ones((P, 1), dtype=dt, device=means3D.device)
    ph = torch.cat([means3D, ones], 1)
    p_view = ph @ view
    p_hom = ph @ proj
    p_w = 1.0 / (p_hom[:, 3:4] + 1e-7)
    ndc = p_hom[:, :2] * p_w + means2D[:, :2]
    if cov3D is None:
        R = quat_R(rots)
        L = R * (mod * scales)[:, None, :]
        Sig = L @ L.transpose(1, 2)
    else:
        c = cov3D
        Sig = torch.stack([torch.stack([c[:, 0], c[:, 1], c[:, 2]], -1), torch.stack([c[:, 1], c[:, 3], c[:, 4]], -1),
                           torch.stack([c[:, 2], c[:, 4], c[:, 5]], -1)], -2)
    fx, fy = W / (2 * tanfovx), H / (2 * tanfovy)
    tz = p_view[:, 2]
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    txtz, tytz = p_view[:, 0] / tz, p_view[:, 1] / tz
    tx = torch.clamp(txtz, -limx, limx) * tz
    ty = torch.clamp(tytz, -limy, limy) * tz
    # upstream's gradient through the clamp: a clamped t.x / t.y is a constant of the Jacobian
    # (x_grad_mul = 0 and no tz term through it), not limx * tz
    tx = torch.where(txtz.abs() > limx, tx.detach(), tx)
    ty = torch.where(tytz.abs() > limy, ty.detach(), ty)
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / tz ** 2], -1),
                     torch.stack([zero, fy / tz, -fy * ty / tz ** 2], -1)], -2)
    Rw = view[:3, :3].T
    T = J @ Rw
    cov2 = T @ Sig @ T.transpose(1, 2)
    a, b, c = cov2[:, 0, 0] + 0.3, cov2[:, 0, 1], cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], -1)
    with torch.no_grad():
        mid = 0.5 * (a + c)
        disc = torch.clamp(mid * mid - det, min=0.1)
        lam = torch.maximum(mid + disc.sqrt(), mid - disc.sqrt())
        radius = torch.ceil(3 * lam.sqrt())
    pix = ((ndc + 1) * torch.tensor([W, H], dtype=dt, device=means3D.device) - 1) * 0.5
    if colors is None:
        d = means3D - campos[None]
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_rgb(deg, shs, d) + 0.5, 0.0)
    else:
        rgb = colors
    gx, gy = (W + 15) // 16, (H + 15) // 16
    with torch.no_grad():
        px_, py_ = pix[:, 0], pix[:, 1]
        x0 = torch.clamp(((px_ - radius) / 16).trunc(), 0, gx)
        y0 = torch.clamp(((py_ - radius) / 16).trunc(), 0, gy)
        x1 = torch.clamp(((px_ + radius + 15) / 16).trunc(), 0, gx)
        y1 = torch.clamp(((py_ + radius + 15) / 16).trunc(), 0, gy)
        visible = (tz > 0.2) & (det != 0) & ((x1 - x0) * (y1 - y0) > 0)
        radii = torch.where(visible, radius, torch.zeros_like(radius)).to(torch.int32)
        srt = torch.argsort(tz, stable=True)
        order = srt[visible[srt]].tolist()
    return dict(pix=pix, conic=conic, rgb=rgb, tz=tz, x0=x0, y0=y0, x1=x1, y1=y1, radii=radii, order=order)


def render(means3D, means2D, opac, view, proj, campos, tanfovx, tanfovy, W, H, bg, shs=None, deg=0, colors=None,
           scales=None, rots=None, cov3D=None, mod=1.0):
    """Returns (image [3, H, W], radii [P]).  All inputs double precision recommended."""
    dt = means3D.dtype
    q = _prep(means3D, means2D, opac, view, proj, campos, tanfovx, tanfovy, W, H, shs, deg, colors, scales, rots,
              cov3D, mod)
    pix, conic, rgb, x0, y0, x1, y1, radii, order = (q[k] for k in ("pix", "conic", "rgb", "x0", "y0", "x1", "y1",
                                                                     "radii", "order"))
    ys, xs = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    xs, ys = xs.reshape(-1), ys.reshape(-1)
    txi, tyi = (xs // 16), (ys // 16)
    Tr = torch.ones_like(xs)
    C = torch.zeros((3, xs.shape[0]), dtype=dt)
    done = torch.zeros_like(xs, dtype=torch.bool)
    for i in order:
        inrect = (txi >= x0[i]) & (txi < x1[i]) & (tyi >= y0[i]) & (tyi < y1[i])
        dx, dy = pix[i, 0] - xs, pix[i, 1] - ys
        power = -0.5 * (conic[i, 0] * dx * dx + conic[i, 2] * dy * dy) - conic[i, 1] * dx * dy
        G = torch.exp(power)
        a_raw = opac[i] * G
        alpha = a_raw - torch.clamp(a_raw.detach() - 0.99, min=0.0)   # min(0.99, .) with straight-through grad
        with torch.no_grad():
            ok = inrect & ~done & (power <= 0) & (alpha >= 1.0 / 255.0)
            test_T = Tr * (1 - alpha)
            stop = ok & (test_T < 1e-4)
            ok = ok & ~stop
            done = done | stop
        okf = ok.to(dt)
        C = C + rgb[i][:, None] * (alpha * Tr * okf)[None]
        Tr = torch.where(ok, Tr * (1 - alpha), Tr)
    img = C + Tr[None] * bg[:, None]
    return img.reshape(3, H, W), radii


def render_local(means3D, means2D, opac, view, proj, campos, tanfovx, tanfovy, W, H, bg, shs=None, deg=0,
                 colors=None, scales=None, rots=None, cov3D=None, mod=1.0, flag_rel=1e-5, flag_T_rel=None):
    """The same function as render(), composited Gaussian by Gaussian over the pixels of its tile
    rectangle only (gathers / index_add into the flat image), so it runs on a GPU at thousands of
    Gaussians.  Also returns a bool [H, W] map of the pixels where some tested decision lies within
    `flag_rel` (relative) of its threshold -- alpha vs 1/255, the tested T vs 1e-4 (`flag_T_rel`
    if given) -- or power within 1e-6 of 0: there an fp32 evaluation may decide the other way."""
    flag_T_rel = flag_rel if flag_T_rel is None else flag_T_rel
    dt, dev = means3D.dtype, means3D.device
    q = _prep(means3D, means2D, opac, view, proj, campos, tanfovx, tanfovy, W, H, shs, deg, colors, scales, rots,
              cov3D, mod)
    pix, conic, rgb, x0, y0, x1, y1, radii, order = (q[k] for k in ("pix", "conic", "rgb", "x0", "y0", "x1", "y1",
                                                                     "radii", "order"))
    npx = W * H
    Tr = torch.ones(npx, dtype=dt, device=dev)
    C = torch.zeros((3, npx), dtype=dt, device=dev)
    done = torch.zeros(npx, dtype=torch.bool, device=dev)
    flag = torch.zeros(npx, dtype=torch.bool, device=dev)
    rect = torch.stack([x0, y0, x1, y1], 1).to(torch.int64).cpu()
    for i in order:
        rx0, ry0, rx1, ry1 = (int(v) for v in rect[i])
        xs = torch.arange(16 * rx0, min(16 * rx1, W), device=dev)
        ys = torch.arange(16 * ry0, min(16 * ry1, H), device=dev)
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        idx = (yy * W + xx).reshape(-1)
        dx, dy = pix[i, 0] - xx.reshape(-1).to(dt), pix[i, 1] - yy.reshape(-1).to(dt)
        power = -0.5 * (conic[i, 0] * dx * dx + conic[i, 2] * dy * dy) - conic[i, 1] * dx * dy
        a_raw = opac[i] * torch.exp(power)
        alpha = a_raw - torch.clamp(a_raw.detach() - 0.99, min=0.0)   # min(0.99, .), straight-through grad
        Ti = Tr[idx]
        with torch.no_grad():
            live = ~done[idx]
            ok = live & (power <= 0) & (alpha >= 1.0 / 255.0)
            test_T = Ti * (1 - alpha)
            stop = ok & (test_T < 1e-4)
            near = live & (((alpha - 1.0 / 255.0).abs() <= flag_rel / 255.0) | (power.abs() <= 1e-6)
                           | (ok & ((test_T - 1e-4).abs() <= flag_T_rel * 1e-4)))
            flag[idx] |= near
            ok = ok & ~stop
            done[idx] |= stop
        okf = ok.to(dt)
        C = C.index_add(1, idx, rgb[i][:, None] * (alpha * Ti * okf)[None])
        Tr = Tr.index_put((idx,), torch.where(ok, Ti * (1 - alpha), Ti))
    img = C + Tr[None] * bg[:, None]
    return img.reshape(3, H, W), radii, flag.reshape(H, W)
