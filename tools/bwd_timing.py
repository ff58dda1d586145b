"""Critical path of k_render_bwd_tw: per-wave start / end stamps of one backward launch.

Needs a library built with -DGS_TIMING (make -C gaussian-splatting-skysphere_amd BUILD=build_timing
EXTRA=-DGS_TIMING) and GSRAST_LIB pointing at it.  Runs the batch-1 loop (bench.py's single_view
shape), then one more iteration with the stamp buffer cleared, and reports: the launch's span against
its longest wave, the resident-wave profile over time, the tail, per-XCD spans, and how a wave's
duration follows its walk (entries walked, slots evaluated).  The stamps are s_memrealtime (100 MHz).
"""
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
ap.add_argument("--reps", type=int, default=3, help="stamped launches (each one iteration after warm-up)")
ap.add_argument("--out", default="")
ap.add_argument("--raw", default="", help="also save the per-wave arrays of the last launch (npz)")
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
lib.gs_debug_bwd_timing.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
lib.gs_debug_bwd_timing.restype = ctypes.c_int


def step():
    bucket.zero_grad()
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3], rotations=params[4])
    img.backward(dpix)
    bucket.finalize()


for _ in range(20):
    step()
torch.cuda.synchronize()
gx, gy = (W + 15) // 16, (H + 15) // 16
tiles = gx * gy
slots = 8 * ((tiles + 7) // 8) + 8
reports = []
for rep in range(a.reps):
    assert lib.gs_debug_bwd_timing(None, 0, 1) == 0
    lib.gs_profile_reset()
    lib.gs_profile_enable(1)
    step()
    torch.cuda.synchronize()
    lib.gs_profile_enable(0)
    ev_us = 1e3 * _native.profile_stats()["render_bwd"][0]
    buf = (ctypes.c_ulonglong * (slots * 5))()
    assert lib.gs_debug_bwd_timing(buf, slots, 0) == 0
    d = np.frombuffer(buf, dtype=np.uint64).reshape(slots, 5)
    d = d[d[:, 1] != 0]
    t0 = d[:, 0].astype(np.int64)
    t1 = d[:, 1].astype(np.int64)
    base = t0.min()
    s_us = (t0 - base) / 100.0  # 100 MHz -> us
    e_us = (t1 - base) / 100.0
    dur = e_us - s_us
    n_eff = (d[:, 2] & 0xFFFFFFFF).astype(np.int64)
    walked = (d[:, 4] >> 32).astype(np.int64)
    nslots = (d[:, 4] & 0xFFFFFFFF).astype(np.int64)
    xcc = (d[:, 3] >> 32).astype(np.int64) & 0xF
    hw = (d[:, 3] & 0xFFFFFFFF).astype(np.int64)
    span = e_us.max()
    il = int(np.argmax(dur))
    order = np.argsort(dur)[::-1]
    # resident waves over time (1 us bins)
    nb = int(np.ceil(span)) + 1
    occ = np.zeros(nb)
    for s, e in zip(s_us, e_us):
        occ[int(s):int(np.ceil(e))] += 1
    # least-squares duration model: a + b walked + c slots
    X = np.stack([np.ones_like(dur), walked, nslots], 1)
    coef, *_ = np.linalg.lstsq(X, dur, rcond=None)
    active = walked > 0
    # per-XCD spans
    per_xcd = {}
    for x in range(8):
        m = xcc == x
        if m.any():
            per_xcd[int(x)] = {"waves": int(m.sum()), "first_start": round(float(s_us[m].min()), 1),
                               "last_end": round(float(e_us[m].max()), 1), "sum_dur": round(float(dur[m].sum()), 0),
                               "entries": int(walked[m].sum())}
    # SIMD / CU identity (gfx9 HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    sh = (hw >> 12) & 1
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simd_key = cu_key * 4 + simd
    simd_busy_end = {}
    for k, e in zip(simd_key, e_us):
        simd_busy_end[int(k)] = max(simd_busy_end.get(int(k), 0.0), float(e))
    ends = np.array(sorted(simd_busy_end.values()))
    # waves still running at fractions of the span
    frac_run = {f"{f:.1f}": int(((s_us <= f * span) & (e_us > f * span)).sum()) for f in (0.5, 0.7, 0.8, 0.9, 0.95)}
    rep_d = {
        "workload": a.workload, "rep": rep, "event_us": round(ev_us, 1), "span_us": round(float(span), 1),
        "waves": int(len(dur)), "waves_with_walk": int(active.sum()), "simds_seen": int(len(simd_busy_end)),
        "longest_wave_us": round(float(dur[il]), 1), "longest_over_span": round(float(dur[il] / span), 3),
        "longest_wave": {"n_eff": int(n_eff[il]), "walked": int(walked[il]), "slots": int(nslots[il]),
                         "start_us": round(float(s_us[il]), 1), "xcc": int(xcc[il])},
        "top10_dur_us": [round(float(dur[i]), 1) for i in order[:10]],
        "top10_walked": [int(walked[i]) for i in order[:10]],
        "top10_start_us": [round(float(s_us[i]), 1) for i in order[:10]],
        "dur_pct": {p: round(float(np.percentile(dur[active], p)), 1) for p in (10, 50, 90, 99)},
        "walked_pct": {p: int(np.percentile(walked[active], p)) for p in (10, 50, 90, 99)},
        "max_walked": int(walked.max()), "mean_walked": round(float(walked[active].mean()), 1),
        "last_start_us": round(float(s_us.max()), 1),
        "model_us": {"const": round(float(coef[0]), 2), "per_entry": round(float(coef[1]), 4),
                     "per_slot": round(float(coef[2]), 4)},
        "resident_waves_by_10pct": [round(float(occ[int(i * nb / 10):int((i + 1) * nb / 10)].mean()), 0)
                                    for i in range(10)],
        "running_at_frac_of_span": frac_run,
        "simd_last_end_pct_of_span": {p: round(float(np.percentile(ends, p) / span), 3) for p in (5, 25, 50, 75, 95)},
        "per_xcd": per_xcd,
    }
    reports.append(rep_d)
    if a.raw:
        np.savez(a.raw, start_us=s_us, end_us=e_us, tile=(d[:, 2] >> 32).astype(np.int64), n_eff=n_eff, walked=walked,
                 slots=nslots, xcc=xcc, simd_key=simd_key, launch_pos=np.nonzero(np.asarray(
                     np.frombuffer(buf, dtype=np.uint64).reshape(slots, 5)[:, 1] != 0))[0])
    print(json.dumps(rep_d), flush=True)
if a.out:
    with open(a.out, "w") as f:
        json.dump(reports, f, indent=1)
