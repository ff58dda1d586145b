"""Tile-exact binning is output-preserving: with the instance list cut to the
tiles whose pixels the alpha >= 1/255 ellipse can reach, the oracle's image, radii and every
gradient are bit-identical to binning into the full upstream tile rectangle, while the instance
count drops."""
import math

import numpy as np
import pytest

import gs_scenes


def _scene(oracle, P, deg, W, H, seed):
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=seed)
    return oracle.Scene(bg=np.array([0.2, 0.5, 0.1], np.float32), means3D=sc.means3D.numpy(),
                        opacities=sc.opacities.numpy(), W=W, H=H, viewmatrix=cam.world_view_transform.numpy(),
                        projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                        tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2), shs=sc.shs.numpy(),
                        sh_degree=deg, scales=sc.scales.numpy(), rotations=sc.rotations.numpy())


@pytest.mark.parametrize("P,deg,W,H,seed", [(3000, 1, 203, 117, 3), (20000, 3, 320, 240, 4)])
def test_exact_tiles_preserve_outputs(oracle, P, deg, W, H, seed):
    sc = _scene(oracle, P, deg, W, H, seed)
    dpix = gs_scenes.dl_dimage(H, W, seed=1).numpy()
    try:
        oracle.set_exact_tiles(False)
        f_rect = oracle.forward(sc)
        b_rect = oracle.backward(sc, dpix)
        oracle.set_exact_tiles(True)
        f_ex = oracle.forward(sc)
        b_ex = oracle.backward(sc, dpix)
    finally:
        oracle.set_exact_tiles(True)
    assert f_ex["num_rendered"] < f_rect["num_rendered"]
    np.testing.assert_array_equal(f_ex["color"], f_rect["color"])
    np.testing.assert_array_equal(f_ex["radii"], f_rect["radii"])
    for k in ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dsh", "dscales", "drotations", "dconic"):
        np.testing.assert_array_equal(b_ex[k], b_rect[k], err_msg=k)
