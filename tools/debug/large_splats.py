"""Debug: per-Gaussian GPU vs oracle gradient comparison for the large/elongated splat scene."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np, torch
import gs_scenes
from oracle import gs_oracle as oracle
from test_gpu_parity import _oracle_scene, _gpu_run
dev = torch.device("cuda:0")
W, H = 640, 360
cam = gs_scenes.identity_camera(W, H)
small = gs_scenes.random_gaussians(3000, 2, cam=cam, seed=21)
big = gs_scenes.random_gaussians(60, 2, cam=cam, seed=22, scale_range=(0.05, 1.5), z_range=(2.0, 4.0))
big.scales[::3, 0] *= float(sys.argv[1]) if len(sys.argv) > 1 else 0.2
sc = gs_scenes.concat_scenes(small, big)
bg = np.array([0.1, 0.2, 0.3], np.float32)
osc = _oracle_scene(oracle, cam, sc, bg)
ofw = oracle.forward(osc, intermediates=True)
dpix = gs_scenes.dl_dimage(H, W, seed=23).numpy()
img, _, leaves = _gpu_run(cam, sc, dev, bg, dpix)
gr = oracle.backward(osc, dpix)
g = {k: v.grad.detach().cpu().numpy() for k, v in leaves.items()}
ref = gr["dmeans3D"]; got = g["means3D"]
d = np.abs(got - ref)
tol = 1e-5 * np.abs(ref) + 1e-5 * np.abs(ref).max()
bad = np.unique(np.nonzero(d > tol)[0])
print("bad gaussians", bad, "of", sc.P)
for i in bad:
    print(f"i={i} tiles={ofw['tiles_touched'][i]} r={ofw['radii'][i]} scales={sc.scales[i].numpy()} op={sc.opacities[i].item():.3f}")
    print("  dmeans3D gpu", got[i], "ref", ref[i])
    for k, rk in (("means2D", "dmeans2D"), ("opacities", "dopacity"), ("scales", "dscales"), ("rotations", "drotations")):
        print(f"  {k:10s} gpu {g[k][i]} ref {gr[rk][i]}")
    print("  dsh rel err", np.abs(g['shs'][i] - gr['dsh'][i]).max() / max(np.abs(gr['dsh'][i]).max(), 1e-30))
    print("  dconic ref", gr["dconic"][i].ravel())
