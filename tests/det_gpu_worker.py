"""Worker of tests/test_gpu_multiview.py::test_concurrent_processes_are_deterministic: renders the
8 C4 ring views (1M Gaussians in a ball) forward + backward, then again `reps` times, and compares
every image and gradient bitwise with the first pass.  Two of these run at once on one GPU (the
timing that exposed a missing LDS drain before a workgroup barrier, gs_common.h lds_barrier).
Prints "OK ..." or "FAIL ..." and exits non-zero on a difference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402

import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

W, H = 1920, 1080
NAMES = ("img", "means3D", "shs", "opacities", "scales", "rotations", "means2D")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    cams = gs_scenes.circle_cameras(8, 6.0, W, H)
    d = gs_scenes.random_gaussians(1_000_000, 3, seed=0, ball_radius=2.0).to(dev)
    dl = [gs_scenes.dl_dimage(H, W, seed=100 + v).to(dev) for v in range(8)]

    def view(v):
        p = [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True),
             d.opacities.clone().requires_grad_(True), d.scales.clone().requires_grad_(True),
             d.rotations.clone().requires_grad_(True)]
        m2 = torch.zeros_like(p[0], requires_grad=True)
        rast = GaussianRasterizer(gs_scenes.raster_settings_for(cams[v], 3, device=dev))
        img, _ = rast(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4])
        img.backward(dl[v])
        return [img.detach()] + [x.grad for x in p] + [m2.grad]

    ref = [view(v) for v in range(8)]
    bad = []
    for r in range(reps):
        for v in range(8):
            for name, a, b in zip(NAMES, view(v), ref[v]):
                if not torch.equal(a, b):
                    bad.append(f"rep {r} view {v} {name}: {int((a != b).sum())} elements")
    torch.cuda.synchronize()
    print(("FAIL " + "; ".join(bad[:10])) if bad else f"OK {reps} reps x 8 views bitwise identical", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
