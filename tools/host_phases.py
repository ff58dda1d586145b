"""Wall time of each host phase of bench.py's multi-view step (fused front, K views on 2 streams,
backwards into a deferred GradBucket): prepare_views, every view's forward and backward call,
finalize.  Steps start from an idle device (synchronised before each), so the times are the host's
own work plus any host wait inside the phase (prepare_views waits for the views' counts).
    python tools/host_phases.py [--workload c2] [--steps 300]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GS_PKG: another copy of the package (an A/B of host-side changes in one call)
sys.path[:0] = [os.environ.get("GS_PKG", os.path.join(ROOT, "gaussian-splatting-skysphere_amd")), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, prepare_views  # noqa: E402

WL = {"c1": (10_000, 0, 256, 256), "c2": (100_000, 3, 800, 800)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=sorted(WL))
ap.add_argument("--steps", type=int, default=300)
ap.add_argument("--views", type=int, default=4)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--ab", action="store_true",
                help="alternate blocks with the round-4 host changes undone in process (ctypes per-Gaussian "
                     "pass, fresh events per deferred view, torch.cuda.stream) against this tree")
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
cams = gs_scenes.jittered_cameras(a.views, W, H, seed=7)
cams[0] = cam
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
dpix = gs_scenes.dl_dimage(H, W, seed=1).to(dev)
rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, deg, device=dev)) for c in cams]
bucket = vp.GradBucket(params, lazy_zero=True, defer=True, chunks=1)
streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
names = ["zero_grad", "prepare_views"] + [f"v{k} {p}" for k in range(a.views) for p in ("fwd", "bwd")] + [
    "finalize"]
acc = dict.fromkeys(names, 0.0)
pc = time.perf_counter


def step(tm):
    t = pc()
    bucket.zero_grad()
    t1 = pc()
    tm["zero_grad"] += t1 - t
    pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4],
                        streams=[streams[k % len(streams)] for k in range(len(rasts))])
    t2 = pc()
    tm["prepare_views"] += t2 - t1
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    for k, (r, p) in enumerate(zip(rasts, pre)):
        with (torch.cuda.stream(streams[k % len(streams)]) if OLD[0] else
              vp._on_stream(streams[k % len(streams)], main)):
            t3 = pc()
            m2 = torch.empty_like(params[0], requires_grad=True)
            img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                       rotations=params[4], prepared=p)
            t4 = pc()
            img.backward(dpix)
            t5 = pc()
            tm[f"v{k} fwd"] += t4 - t3
            tm[f"v{k} bwd"] += t5 - t4
    for s in streams:
        main.wait_stream(s)
    t6 = pc()
    bucket.finalize()
    tm["finalize"] += pc() - t6


OLD = [False]
if a.ab:
    from diff_gaussian_rasterization import _C

    _bwdg = _C.backward_gaussians

    def _bwdg_ctypes(*args, **kw):
        e, _C._EXT = _C._EXT, None
        try:
            return _bwdg(*args, **kw)
        finally:
            _C._EXT = e

    class _NoPool(list):
        def __iadd__(self, other):
            return self

    def set_mode(old):
        OLD[0] = old
        _C.backward_gaussians = _bwdg_ctypes if old else _bwdg
        bucket._ev_pool = _NoPool() if old else []

    import statistics
    res = {m: {"b2b": [], "idle": [], **{n: [] for n in names}} for m in ("new", "old")}
    for _ in range(20):
        step(dict(acc))
    for blk in range(16):
        m = "old" if blk % 2 else "new"
        set_mode(m == "old")
        for _ in range(10):
            step(dict(acc))
        torch.cuda.synchronize()
        t0 = pc()
        for _ in range(50):
            step(dict(acc))
        torch.cuda.synchronize()
        res[m]["b2b"].append((pc() - t0) / 50)
        tm = dict.fromkeys(names, 0.0)
        tot = 0.0
        for _ in range(50):
            torch.cuda.synchronize()
            t = pc()
            step(tm)
            tot += pc() - t
        res[m]["idle"].append(tot / 50)
        for n in names:
            res[m][n].append(tm[n] / 50)
    torch.cuda.synchronize()
    print("median over 8 alternating blocks of 50 steps (us)    new     old")
    for k in ["b2b", "idle"] + names:
        print(f"  {k:14s} {1e6 * statistics.median(res['new'][k]):8.1f} {1e6 * statistics.median(res['old'][k]):8.1f}")
    sys.exit(0)

for _ in range(20):
    step(dict(acc))
torch.cuda.synchronize()
t0 = pc()
for _ in range(a.steps):
    step(dict(acc))
torch.cuda.synchronize()
dt = (pc() - t0) / a.steps
print(os.environ.get("GS_PKG", "(this tree)"))
print(f"{a.workload} {a.views}-view step back to back: {1e3 * dt:.4f} ms ({a.views / dt:.1f} views/s)")
tot = 0.0
for _ in range(a.steps):
    torch.cuda.synchronize()
    t = pc()
    step(acc)
    tot += pc() - t
torch.cuda.synchronize()
print(f"from an idle device: {1e6 * tot / a.steps:.1f} us of host time per step")
for n in names:
    print(f"  {n:14s} {1e6 * acc[n] / a.steps:8.1f} us")
