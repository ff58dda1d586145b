"""Debug: the bounded view-parallel step in a HIP graph, replayed after in-place parameter changes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), os.path.join(ROOT, "tests"), ROOT]
import torch
import gs_scenes
import gs_view_parallel as vp
from diff_gaussian_rasterization import GaussianRasterizer, bounded_status, last_num_rendered

device = torch.device("cuda:0")
W, H = 320, 240
d = gs_scenes.random_gaussians(20_000, 3, seed=9, ball_radius=2.0).to(device)
cams = gs_scenes.circle_cameras(3, 6.0, W, H)
rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
dpix = [gs_scenes.dl_dimage(H, W, seed=60 + v).to(device) for v in range(3)]
p = [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True), d.opacities.clone().requires_grad_(True),
     d.scales.clone().requires_grad_(True), d.rotations.clone().requires_grad_(True)]
counts = []
with torch.no_grad():
    for r in rasts:
        r(means3D=p[0], means2D=torch.zeros_like(p[0]), opacities=p[2], shs=p[1], scales=p[3], rotations=p[4])
        counts.append(last_num_rendered())
cap = int(max(counts) * 1.25)
print("counts", counts, "cap", cap, "scales", float(d.scales.min()), float(d.scales.max()))
bucket = vp.GradBucket(p, lazy_zero=True, defer=False)
streams = [torch.cuda.Stream(device)]
imgs = [None] * 3

def view(k, r, dp, c):
    def run():
        m2 = torch.empty_like(p[0], requires_grad=True)
        img, _ = r(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4], binning_capacity=c)
        img.backward(dp)
        imgs[k] = img.detach()
    return run

def step(c):
    bucket.zero_grad()
    vp.run_views([view(k, r, dp, c) for k, (r, dp) in enumerate(zip(rasts, dpix))], streams)
    bucket.finalize()

side = torch.cuda.Stream(device)
side.wait_stream(torch.cuda.current_stream(device))
with torch.cuda.stream(side):
    for _ in range(2):
        step(cap)
torch.cuda.current_stream(device).wait_stream(side)
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    step(cap)
graph.replay(); torch.cuda.synchronize()
print("replay0 flat absmax", float(bucket.flat.abs().max()), "status", bounded_status())
gen = torch.Generator(device=device).manual_seed(77)
for it in range(2):
    with torch.no_grad():
        for t in p:
            t.add_(0.02 * torch.randn(t.shape, device=device, generator=gen))
    cs = []
    with torch.no_grad():
        for r in rasts:
            r(means3D=p[0], means2D=torch.zeros_like(p[0]), opacities=p[2], shs=p[1], scales=p[3], rotations=p[4])
            cs.append(last_num_rendered())
    step(None); torch.cuda.synchronize()
    ref = bucket.flat.clone(); ref_imgs = [t.clone() for t in imgs]
    bucket.flat.fill_(float("nan"))
    graph.replay(); torch.cuda.synchronize()
    print("it", it, "counts", cs, "flat nan", int(bucket.flat.isnan().sum()), "absmax", float(bucket.flat.abs().max()),
          "ref absmax", float(ref.abs().max()), "eq", torch.equal(bucket.flat, ref),
          "imgs eq", [torch.equal(a, b) for a, b in zip(imgs, ref_imgs)], "img max", [float(a.max()) for a in imgs])
    try:
        print("status", bounded_status())
    except RuntimeError as e:
        print("status raised", e)
