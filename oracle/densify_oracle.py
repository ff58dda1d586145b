"""Restatement of GaussianModel.densify_and_prune -- TEST INFRASTRUCTURE ONLY.

Follows /root/reference/scene/gaussian_model.py step by step, on any torch device:
  densify_and_prune   :391-403  grads = accum / denom (NaN -> 0); clone; split; prune by opacity and,
                                when max_screen_size is truthy, by max_radii2D (already re-zeroed by the
                                postfix) and world-space size > 0.1 * extent
  densify_and_clone   :375-389  |g| >= thr and max(exp(scaling)) <= percent_dense * extent
  densify_and_split   :348-373  g >= thr (clones padded with 0) and max(exp(scaling)) > percent_dense *
                                extent; N children: xyz = R(q) @ normal(0, exp(s)) + xyz, scaling =
                                log(exp(s) / (0.8 N)), other rows repeated; then the parents pruned
  densification_postfix :328-346 / cat_tensors_to_optimizer :307-326  params and Adam moments
                                extended (moments with zeros), stats re-zeroed
  prune_points / _prune_optimizer :272-305
  build_rotation  utils/general_utils.py:78-100
Pinned against tests/golden/densify_golden.npz, produced by the reference's own GaussianModel on
CPU (tests/golden/make_golden.py).  Only tests/ import this module.

The model is a plain namespace with the reference attribute names (_xyz, _features_dc,
_features_rest, _opacity, _scaling, _rotation, xyz_gradient_accum, denom, max_radii2D,
percent_dense, optimizer with named param groups).
"""
from __future__ import annotations

import torch

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
ATTRS = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")


def rotation_matrices(q: torch.Tensor) -> torch.Tensor:
    """R[P,3,3] from raw quaternions (w, x, y, z), normalised by their norm (general_utils.py:78-100)."""
    n = torch.sqrt(q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1] + q[:, 2] * q[:, 2] + q[:, 3] * q[:, 3])
    u = q / n[:, None]
    w, x, y, z = u[:, 0], u[:, 1], u[:, 2], u[:, 3]
    rows = [
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y),
    ]
    return torch.stack(rows, dim=1).view(-1, 3, 3)


def _swap(model, group, new_param, state_fn):
    """Replace a group's tensor and re-key its Adam state (the reference's optimizer surgery)."""
    opt = model.optimizer
    old = group["params"][0]
    st = opt.state.get(old, None)
    p = torch.nn.Parameter(new_param.requires_grad_(True))
    if st is not None:
        st["exp_avg"] = state_fn(st["exp_avg"])
        st["exp_avg_sq"] = state_fn(st["exp_avg_sq"])
        del opt.state[old]
        opt.state[p] = st
    group["params"][0] = p
    return p


def _append(model, ext: dict):
    for group in model.optimizer.param_groups:
        e = ext[group["name"]]
        p = _swap(model, group, torch.cat((group["params"][0].detach(), e), 0),
                  lambda t, e=e: torch.cat((t, torch.zeros_like(e)), 0))
        setattr(model, ATTRS[NAMES.index(group["name"])], p)
    n = model._xyz.shape[0]
    dev = model._xyz.device
    model.xyz_gradient_accum = torch.zeros((n, 1), device=dev)
    model.denom = torch.zeros((n, 1), device=dev)
    model.max_radii2D = torch.zeros((n,), device=dev)


def _keep(model, keep: torch.Tensor):
    for group in model.optimizer.param_groups:
        p = _swap(model, group, group["params"][0].detach()[keep], lambda t: t[keep])
        setattr(model, ATTRS[NAMES.index(group["name"])], p)
    model.xyz_gradient_accum = model.xyz_gradient_accum[keep]
    model.denom = model.denom[keep]
    model.max_radii2D = model.max_radii2D[keep]


def densify_and_prune(model, max_grad: float, min_opacity: float, extent: float, max_screen_size, N: int = 2):
    dev = model._xyz.device
    g = model.xyz_gradient_accum / model.denom
    g[g.isnan()] = 0.0

    # clone (:375-389)
    s = torch.exp(model._scaling.detach())
    sel = (torch.norm(g, dim=-1) >= max_grad) & (s.max(dim=1).values <= model.percent_dense * extent)
    _append(model, {n: getattr(model, a).detach()[sel] for n, a in zip(NAMES, ATTRS)})

    # split (:348-373)
    P1 = model._xyz.shape[0]
    gp = torch.zeros((P1,), device=dev)
    gp[:g.shape[0]] = g.squeeze()
    s = torch.exp(model._scaling.detach())
    sel = (gp >= max_grad) & (s.max(dim=1).values > model.percent_dense * extent)
    stds = s[sel].repeat(N, 1)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds)
    R = rotation_matrices(model._rotation.detach()[sel]).repeat(N, 1, 1)
    ext = {
        "xyz": torch.bmm(R, samples.unsqueeze(-1)).squeeze(-1) + model._xyz.detach()[sel].repeat(N, 1),
        "scaling": torch.log(s[sel].repeat(N, 1) / (0.8 * N)),
        "rotation": model._rotation.detach()[sel].repeat(N, 1),
        "f_dc": model._features_dc.detach()[sel].repeat(N, 1, 1),
        "f_rest": model._features_rest.detach()[sel].repeat(N, 1, 1),
        "opacity": model._opacity.detach()[sel].repeat(N, 1),
    }
    _append(model, ext)
    drop = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=dev, dtype=torch.bool)))
    _keep(model, ~drop)

    # prune (:394-401)
    prune = (torch.sigmoid(model._opacity.detach()) < min_opacity).squeeze()
    if max_screen_size:
        big_vs = model.max_radii2D > max_screen_size
        big_ws = torch.exp(model._scaling.detach()).max(dim=1).values > 0.1 * extent
        prune = prune | big_vs | big_ws
    _keep(model, ~prune)
