"""Per-iteration train.py work around the rasterizer at 1M Gaussians (SH3) on one GPU, in the
reference's own torch formulation (scene/gaussian_model.py:95-115, 149-163, 405-407;
train.py:86-128): parameter activations + cat, their backward, densification statistics,
Adam step (eps 1e-15, six param groups) and zero_grad.  Prints one JSON line of ms per part."""
import json
import time

import torch

P = 1_000_000
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
xyz = torch.randn((P, 3), generator=g).to(dev).requires_grad_(True)
f_dc = torch.randn((P, 1, 3), generator=g).to(dev).requires_grad_(True)
f_rest = torch.randn((P, 15, 3), generator=g).to(dev).requires_grad_(True)
opac = torch.randn((P, 1), generator=g).to(dev).requires_grad_(True)
scal = torch.randn((P, 3), generator=g).to(dev).requires_grad_(True)
rot = torch.randn((P, 4), generator=g).to(dev).requires_grad_(True)
params = [xyz, f_dc, f_rest, opac, scal, rot]
opt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in
                        zip(params, [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3])], lr=0.0, eps=1e-15)
accum = torch.zeros((P, 1), device=dev)
denom = torch.zeros((P, 1), device=dev)
max_r = torch.zeros((P,), device=dev)
radii = torch.randint(0, 20, (P,), device=dev, dtype=torch.int32)
m2d = torch.zeros((P, 3), device=dev, requires_grad=True)


def act():
    return (xyz, torch.cat((f_dc, f_rest), 1), torch.sigmoid(opac), torch.exp(scal),
            torch.nn.functional.normalize(rot))


def timeit(fn, steps=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


grads = [torch.randn_like(t) for t in act()]


def fwd_bwd():
    outs = act()
    torch.autograd.backward(outs[1:], grads[1:])


def densify_stats():
    vis = radii > 0
    max_r[vis] = torch.max(max_r[vis], radii[vis].float())
    m2d.grad = torch.randn_like(m2d)
    accum[vis] += torch.norm(m2d.grad[vis, :2], dim=-1, keepdim=True)
    denom[vis] += 1


for p in params:
    p.grad = torch.randn_like(p)


def adam():
    opt.step()


def zero():
    opt.zero_grad(set_to_none=True)
    for p in params:
        p.grad = torch.zeros_like(p)


r = {"activations_fwd_bwd_ms": timeit(fwd_bwd), "densify_stats_ms": timeit(densify_stats),
     "adam_step_ms": timeit(adam)}

# the fused HIP versions (gs_train) on the same tensors
import sys, os  # noqa: E401,E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gaussian-splatting-skysphere_amd"))
import gs_train  # noqa: E402

fopt = gs_train.FusedAdam([{"params": [p], "lr": lr} for p, lr in
                           zip(params, [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3])], lr=0.0, eps=1e-15)
m2d.grad = torch.randn_like(m2d)


def fused_densify():
    gs_train.densify_stats(max_r, accum, denom, radii, m2d.grad)


def fused_fwd_bwd():
    outs = gs_train.activate(f_dc, f_rest, opac, scal, rot)
    torch.autograd.backward(outs, grads[1:])


r["fused_activations_fwd_bwd_ms"] = timeit(fused_fwd_bwd)
r["fused_adam_step_ms"] = timeit(fopt.step)
r["fused_densify_stats_ms"] = timeit(fused_densify)
# device-only time of the fused Adam launch (host-side Python excluded) via events
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    fopt.step()
e1.record()
torch.cuda.synchronize()
r["fused_adam_step_events_ms"] = e0.elapsed_time(e1) / 20
nbytes = sum(p.numel() for p in params) * 4 * 7  # read p, g, m, v; write p, m, v
r["fused_adam_GBps"] = nbytes / (r["fused_adam_step_events_ms"] * 1e-3) / 1e9



# ---- densify_and_prune at 1M: the reference's torch sequence (gaussian_model.py:258-403: clone cat,
# split cat, parent prune, final prune, each rewriting params + Adam moments) vs gs_train's 3 passes
class _M:
    pass


def _densify_model(P, seed=0):
    import math
    gg = torch.Generator().manual_seed(seed)
    m = _M()
    m.percent_dense = 0.01
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    attrs = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
    groups = []
    for (n, sh), a in zip(shapes.items(), attrs):
        t = torch.randn(sh, generator=gg)
        if n == "scaling":
            t = math.log(0.003) + torch.rand(sh, generator=gg) * (math.log(0.5) - math.log(0.003))
        p = torch.nn.Parameter(t.to(dev))
        setattr(m, a, p)
        groups.append({"params": [p], "lr": 1e-3, "name": n})
    m.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    for grp in m.optimizer.param_groups:
        p = grp["params"][0]
        m.optimizer.state[p] = {"step": torch.tensor(10.0), "exp_avg": torch.randn_like(p) * 1e-3,
                                "exp_avg_sq": torch.rand_like(p) * 1e-6}
    m.denom = torch.randint(0, 4, (P, 1), generator=gg).float().to(dev)
    # about 5% of the Gaussians cross the gradient threshold (clone or split)
    m.xyz_gradient_accum = (torch.rand((P, 1), generator=gg) * 2.1e-4 * m.denom.cpu()).to(dev)
    m.max_radii2D = torch.zeros((P,), device=dev)
    return m, attrs


def _torch_densify(m, attrs, max_grad=2e-4, min_opacity=0.005, extent=2.0, max_screen_size=20, N=2):
    names = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")

    def swap(new_fn, state_fn):
        for grp in m.optimizer.param_groups:
            old = grp["params"][0]
            st = m.optimizer.state.pop(old)
            st["exp_avg"], st["exp_avg_sq"] = state_fn(st["exp_avg"], grp), state_fn(st["exp_avg_sq"], grp)
            p = torch.nn.Parameter(new_fn(old.detach(), grp).requires_grad_(True))
            m.optimizer.state[p] = st
            grp["params"][0] = p
            setattr(m, attrs[names.index(grp["name"])], p)

    def cat(ext):
        swap(lambda t, grp: torch.cat((t, ext[grp["name"]]), 0),
             lambda t, grp: torch.cat((t, torch.zeros_like(ext[grp["name"]])), 0))
        n = m._xyz.shape[0]
        m.xyz_gradient_accum = torch.zeros((n, 1), device=dev)
        m.denom = torch.zeros((n, 1), device=dev)
        m.max_radii2D = torch.zeros((n,), device=dev)

    def keep(mask):
        swap(lambda t, grp: t[mask], lambda t, grp: t[mask])
        m.xyz_gradient_accum, m.denom, m.max_radii2D = m.xyz_gradient_accum[mask], m.denom[mask], m.max_radii2D[mask]

    grads = m.xyz_gradient_accum / m.denom
    grads[grads.isnan()] = 0.0
    s = torch.exp(m._scaling)
    sel = (torch.norm(grads, dim=-1) >= max_grad) & (s.max(1).values <= m.percent_dense * extent)
    cat({n: getattr(m, a).detach()[sel] for n, a in zip(names, attrs)})
    P1 = m._xyz.shape[0]
    pg = torch.zeros((P1,), device=dev)
    pg[:grads.shape[0]] = grads.squeeze()
    s = torch.exp(m._scaling.detach())
    sel = (pg >= max_grad) & (s.max(1).values > m.percent_dense * extent)
    stds = s[sel].repeat(N, 1)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds)
    q = m._rotation.detach()[sel]
    q = q / q.norm(dim=1, keepdim=True)
    w, x, y, z = q.unbind(1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).view(-1, 3, 3)
    cat({"xyz": torch.bmm(R.repeat(N, 1, 1), samples.unsqueeze(-1)).squeeze(-1) + m._xyz.detach()[sel].repeat(N, 1),
         "scaling": torch.log(s[sel].repeat(N, 1) / (0.8 * N)),
         "rotation": m._rotation.detach()[sel].repeat(N, 1), "f_dc": m._features_dc.detach()[sel].repeat(N, 1, 1),
         "f_rest": m._features_rest.detach()[sel].repeat(N, 1, 1), "opacity": m._opacity.detach()[sel].repeat(N, 1)})
    keep(~torch.cat((sel, torch.zeros(N * int(sel.sum()), device=dev, dtype=torch.bool))))
    prune = (torch.sigmoid(m._opacity.detach()) < min_opacity).squeeze()
    if max_screen_size:
        prune = prune | (m.max_radii2D > max_screen_size) | (torch.exp(m._scaling.detach()).max(1).values > 0.1 * extent)
    keep(~prune)


def time_densify(fn, reps=3):
    ts = []
    for r in range(reps + 1):
        m, attrs = _densify_model(P, seed=r)
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        t = time.perf_counter()
        fn(m, attrs)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t) * 1e3)
        peak = (torch.cuda.max_memory_allocated() - base) / 2**20
        out_P = m._xyz.shape[0]
        del m
    return sorted(ts)[len(ts) // 2], peak, out_P


r["densify_and_prune_ms"], r["densify_and_prune_extra_peak_MiB"], r["densify_out_P"] = time_densify(_torch_densify)
r["fused_densify_and_prune_ms"], r["fused_densify_and_prune_extra_peak_MiB"], r["fused_densify_out_P"] = time_densify(
    lambda m, attrs: gs_train.densify_and_prune(m, 2e-4, 0.005, 2.0, 20))
print(json.dumps({k: round(v, 4) for k, v in r.items()}))
