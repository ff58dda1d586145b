"""Critical path of the forward render (k_render_fwd_q): per quadrant-wave start / end stamps.

Needs a library built with -DGS_TIMING (make -C gaussian-splatting-skysphere_amd BUILD=build_timing
EXTRA=-DGS_TIMING) and GSRAST_LIB pointing at it.  Runs the batch-1 loop (bench.py's single_view
shape), then stamped iterations, and reports the launch's span, the resident waves over time, when
the last waves start and how long waves last (by batches staged and entries walked)."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _native  # noqa: E402

WL = {"c3": (1_000_000, 3, 1920, 1080), "c2": (100_000, 3, 800, 800), "c5": (5_000_000, 3, 1920, 1080)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--out", default="")
ap.add_argument("--raw", default="", help="also write each rep's per-wave arrays to RAW.<rep>.npz")
a = ap.parse_args()
P, deg, W, H = WL[a.workload]
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(W, H)
sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0).to(dev)
params = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
bucket = vp.GradBucket(params, lazy_zero=True, defer=False)
dpix = gs_scenes.dl_dimage(H, W).to(dev)
r = GaussianRasterizer(gs_scenes.raster_settings_for(cam, deg, device=dev))
lib = _native.load()
lib.gs_debug_fwd_timing.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
lib.gs_debug_fwd_timing.restype = ctypes.c_int


def step():
    bucket.zero_grad()
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4])
    img.backward(dpix)
    bucket.finalize()


for _ in range(20):
    step()
torch.cuda.synchronize()
slots = 1 << 16
reports = []
for rep in range(a.reps):
    assert lib.gs_debug_fwd_timing(None, 0, 1) == 0
    lib.gs_profile_reset()
    lib.gs_profile_enable(1)
    step()
    torch.cuda.synchronize()
    lib.gs_profile_enable(0)
    ev_us = 1e3 * _native.profile_stats()["render_fwd"][0]
    buf = (ctypes.c_ulonglong * (slots * 5))()
    assert lib.gs_debug_fwd_timing(buf, slots, 0) == 0
    d = np.frombuffer(buf, dtype=np.uint64).reshape(slots, 5)
    d = d[d[:, 1] != 0]
    t0 = d[:, 0].astype(np.int64)
    t1 = d[:, 1].astype(np.int64)
    base = t0.min()
    s_us = (t0 - base) / 100.0
    e_us = (t1 - base) / 100.0
    dur = e_us - s_us
    if a.raw:
        np.savez_compressed(f"{a.raw}.{rep}.npz", start=s_us, end=e_us, tile=(d[:, 2] >> 32).astype(np.int64),
                            quad=(d[:, 2] & 3).astype(np.int64), n=((d[:, 2] & 0xFFFFFFFF) >> 2).astype(np.int64),
                            batches=(d[:, 4] >> 32).astype(np.int64), walked=(d[:, 4] & 0xFFFFFFFF).astype(np.int64),
                            xcc=(d[:, 3] >> 32).astype(np.int64), hw=(d[:, 3] & 0xFFFFFFFF).astype(np.int64))
    batches = (d[:, 4] >> 32).astype(np.int64)
    walked = (d[:, 4] & 0xFFFFFFFF).astype(np.int64)
    span = e_us.max()
    nb = int(np.ceil(span)) + 1
    occ = np.zeros(nb)
    for s, e in zip(s_us, e_us):
        occ[int(s):int(np.ceil(e))] += 1
    X = np.stack([np.ones_like(dur), batches, walked], 1)
    coef, *_ = np.linalg.lstsq(X, dur, rcond=None)
    rep_d = {
        "workload": a.workload, "rep": rep, "event_us": round(ev_us, 1), "span_us": round(float(span), 1),
        "waves": int(len(dur)), "max_resident": int(occ.max()),
        "last_start_us": round(float(s_us.max()), 1), "longest_wave_us": round(float(dur.max()), 1),
        "dur_pct": {p: round(float(np.percentile(dur, p)), 1) for p in (10, 50, 90, 99)},
        "batches_pct": {p: int(np.percentile(batches, p)) for p in (10, 50, 90, 99)},
        "walked_pct": {p: int(np.percentile(walked, p)) for p in (10, 50, 90, 99)},
        "model_us": {"const": round(float(coef[0]), 2), "per_batch": round(float(coef[1]), 3),
                     "per_entry": round(float(coef[2]), 4)},
        "resident_waves_by_10pct": [round(float(occ[int(i * nb / 10):int((i + 1) * nb / 10)].mean()), 0)
                                    for i in range(10)],
        "starts_by_10pct": [int(((s_us >= i * span / 10) & (s_us < (i + 1) * span / 10)).sum()) for i in range(10)],
    }
    reports.append(rep_d)
    print(json.dumps(rep_d), flush=True)
if a.out:
    with open(a.out, "w") as f:
        json.dump(reports, f, indent=1)
