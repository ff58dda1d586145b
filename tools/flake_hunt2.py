"""Run-to-run bitwise check of per-view gradients on the C4 ring scene (1M Gaussians in a ball,
8 ring cameras), repeated; run two copies at once to share the GPU.  Usage: flake_hunt2.py reps tag"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(R, "tests"), os.path.join(R, "gaussian-splatting-skysphere_amd"), R):
    sys.path.insert(0, p)
import torch  # noqa: E402
import gs_scenes  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

reps = int(sys.argv[1])
tag = sys.argv[2] if len(sys.argv) > 2 else ""
if len(sys.argv) > 3 and sys.argv[3] == "poison":
    # every uint8 scratch buffer of the rasterizer starts as 0xFF bytes (NaN as f32): a read of
    # anything this call did not write turns into NaN / garbage instead of a stale value
    from diff_gaussian_rasterization import _C as _Cmod

    class _T:
        def __getattr__(self, k):
            return getattr(torch, k)

        @staticmethod
        def empty(*a, **kw):
            t = torch.empty(*a, **kw)
            if kw.get("dtype") == torch.uint8:
                t.fill_(0xFF)
            return t

    _Cmod.torch = _T()
W, H = 1920, 1080
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
bad = 0
names = ("img", "means3D", "shs", "opac", "scales", "rot", "means2D")
for r in range(reps):
    for v in range(8):
        o = view(v)
        for k, (a, b) in enumerate(zip(o, ref[v])):
            if not torch.equal(a, b):
                bad += 1
                m = (a != b)
                rows = torch.nonzero(m.reshape(m.shape[0], -1).any(1)).flatten() if k else torch.nonzero(m.flatten()).flatten()
                print(f"{tag} rep {r} view {v} {names[k]}: {rows.numel()} rows differ, first {rows[:6].tolist()} "
                      f"max|d| {float((a - b).abs().max()):.3e}", flush=True)
    torch.cuda.synchronize()
print(f"{tag} {reps} reps x 8 views, {bad} differing tensors", flush=True)
