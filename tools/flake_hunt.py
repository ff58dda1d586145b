"""Hunt run-to-run differences of the C3 backward under the parity suite's workload mix: C3 fast-mode
forward + backward repeated, with the smaller parity scenes (exact and fast mode) run in between,
every C3 output compared bitwise with the first C3 run.  Reports the differing Gaussians."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(R, "tests"), os.path.join(R, "gaussian-splatting-skysphere_amd"), R):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gs_scenes  # noqa: E402
from test_gpu_parity import _gpu_run  # noqa: E402
from diff_gaussian_rasterization import _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
lib = _native.load()
dev = torch.device("cuda:0")
cam = gs_scenes.identity_camera(1920, 1080)
sc = gs_scenes.random_gaussians(1_000_000, 3, cam=cam, seed=0)
dpix = gs_scenes.dl_dimage(1080, 1920, seed=1).numpy()
small = []
for (P, deg, W, H) in ((10_000, 0, 256, 256), (3000, 1, 203, 117), (100_000, 3, 800, 800), (60_000, 3, 480, 1080)):
    c = gs_scenes.identity_camera(W, H)
    small.append((c, gs_scenes.random_gaussians(P, deg, cam=c, seed=0), gs_scenes.dl_dimage(H, W, seed=1).numpy()))
bg = np.zeros(3, np.float32)


def c3():
    lib.gs_set_exact_exp(0)
    img, radii, lv = _gpu_run(cam, sc, dev, bg, dpix)
    out = {"img": img.detach().cpu()}
    out.update({k: v.grad.detach().cpu() for k, v in lv.items()})
    return out


ref = c3()
bad = 0
for r in range(n):
    for ex in (1, 0):
        lib.gs_set_exact_exp(ex)
        for (c, s, dp) in small:
            _gpu_run(c, s, dev, bg, dp)
    o = c3()
    diff = {k: (o[k] != ref[k]) for k in ref if not torch.equal(o[k], ref[k])}
    if diff:
        bad += 1
        for k, m in diff.items():
            rows = torch.nonzero(m.reshape(m.shape[0], -1).any(1)).flatten() if k != "img" else torch.nonzero(m.flatten())
            print(f"run {r}: {k} differs at {rows.numel()} rows, first {rows[:8].tolist()}, "
                  f"max|d| {float((o[k] - ref[k]).abs().max()):.3e}", flush=True)
    else:
        print(f"run {r}: identical", flush=True)
print(f"{n} runs, {bad} differing", flush=True)
