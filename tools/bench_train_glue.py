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
print(json.dumps({k: round(v, 4) for k, v in r.items()}))
