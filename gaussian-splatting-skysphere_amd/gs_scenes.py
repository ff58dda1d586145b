"""Synthetic scenes and cameras for benchmarks and tests (SURVEY.md §8d "Synthetic inputs").

Camera matrices follow the reference's conventions exactly:
  getWorld2View2 / getProjectionMatrix  -> /root/reference/utils/graphics_utils.py:38-71
  Camera.world_view_transform / projection_matrix / full_proj_transform / camera_center
                                        -> /root/reference/scene/cameras.py:47-57
(znear 0.01, zfar 100, row-vector convention: the tensors are the transposes of the math matrices).
Gaussian parameters follow the reference model's activations (scene/gaussian_model.py:33-41,
95-115): opacity = sigmoid, scale = exp, rotation = normalize, shs = cat(f_dc, f_rest).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

SH_C0 = 0.28209479177387814


def getWorld2View2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    C2W[:3, 3] = (C2W[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(C2W))


def getProjectionMatrix(znear, zfar, fovX, fovY):
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


@dataclass
class MiniCamera:
    """The camera fields the render adapter reads (gaussian_renderer/__init__.py:33-47)."""

    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor
    projection_matrix: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor

    def to(self, device):
        return MiniCamera(self.image_width, self.image_height, self.FoVx, self.FoVy,
                          self.world_view_transform.to(device), self.projection_matrix.to(device),
                          self.full_proj_transform.to(device), self.camera_center.to(device))


def make_camera(R, T, W, H, fovy_deg=60.0, znear=0.01, zfar=100.0) -> MiniCamera:
    """R: camera-to-world rotation as stored by the reference loaders (transpose of W2C), T: W2C translation."""
    fovy = math.radians(fovy_deg)
    fovx = 2.0 * math.atan(math.tan(fovy / 2.0) * W / H)
    wvt = torch.tensor(getWorld2View2(np.asarray(R, np.float64), np.asarray(T, np.float64))).transpose(0, 1)
    proj = getProjectionMatrix(znear=znear, zfar=zfar, fovX=fovx, fovY=fovy).transpose(0, 1)
    full = (wvt.unsqueeze(0).bmm(proj.unsqueeze(0))).squeeze(0)
    center = wvt.inverse()[3, :3]
    return MiniCamera(W, H, fovx, fovy, wvt, proj, full, center)


def identity_camera(W, H, fovy_deg=60.0) -> MiniCamera:
    return make_camera(np.eye(3), np.zeros(3), W, H, fovy_deg)


def look_at_camera(position, target, W, H, fovy_deg=60.0, up=(0.0, -1.0, 0.0)) -> MiniCamera:
    """OpenCV/COLMAP camera axes (x right, y down, z forward) looking from `position` at `target`."""
    c = np.asarray(position, np.float64)
    f = np.asarray(target, np.float64) - c
    f /= np.linalg.norm(f)
    r = np.cross(f, np.asarray(up, np.float64))
    if np.linalg.norm(r) < 1e-8:
        r = np.cross(f, np.array([1.0, 0.0, 0.0]))
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    w2c = np.stack([r, d, f], axis=0)  # rows: camera axes in world coordinates
    T = -w2c @ c
    return make_camera(w2c.T, T, W, H, fovy_deg)


def jittered_cameras(n, W, H, seed=7, max_angle_deg=2.0, max_shift=0.05, fovy_deg=60.0):
    """n distinct views around the single-view pose: view 0 is identity_camera, view k > 0 is turned
    by a random rotation of up to `max_angle_deg` about a random axis and moved by up to `max_shift`
    along each axis (a batch of nearby training views of one frustum-filled scene)."""
    rng = np.random.default_rng(seed)
    cams = [identity_camera(W, H, fovy_deg)]
    for _ in range(1, n):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        a = math.radians(max_angle_deg) * rng.uniform(0.5, 1.0)
        K = np.array([[0.0, -ax[2], ax[1]], [ax[2], 0.0, -ax[0]], [-ax[1], ax[0], 0.0]])
        w2c = np.eye(3) + math.sin(a) * K + (1.0 - math.cos(a)) * (K @ K)  # Rodrigues
        T = rng.uniform(-max_shift, max_shift, size=3)
        cams.append(make_camera(w2c.T, T, W, H, fovy_deg))
    return cams


def circle_cameras(n, radius, W, H, height=0.0, fovy_deg=60.0):
    """C4: n cameras on a circle of `radius` around the origin, looking at the centre."""
    cams = []
    for v in range(n):
        a = 2.0 * math.pi * v / n
        cams.append(look_at_camera((radius * math.cos(a), height, radius * math.sin(a)), (0.0, 0.0, 0.0), W, H,
                                   fovy_deg))
    return cams


@dataclass
class GaussianScene:
    means3D: torch.Tensor      # [P, 3]
    opacities: torch.Tensor    # [P, 1] (activated)
    scales: torch.Tensor       # [P, 3] (activated)
    rotations: torch.Tensor    # [P, 4] (normalised, w x y z)
    shs: torch.Tensor          # [P, K, 3]
    sh_degree: int

    @property
    def P(self):
        return self.means3D.shape[0]

    def to(self, device):
        return GaussianScene(*(getattr(self, f).to(device) for f in
                               ("means3D", "opacities", "scales", "rotations", "shs")), self.sh_degree)


def random_gaussians(P, sh_degree, cam: MiniCamera | None = None, seed=0, ball_radius=None,
                     scale_range=(0.005, 0.03), z_range=(2.0, 10.0)) -> GaussianScene:
    """means uniform in the view frustum of `cam` (z ~ U(2, 10), x/z, y/z ~ U(-tan, tan)),
    or uniform in a ball of `ball_radius` (C4); log-uniform scales; random unit quaternions;
    sigmoid(N(0,1)) opacity; f_dc = RGB2SH(U(0,1)), f_rest ~ N(0, 0.05^2)."""
    g = torch.Generator().manual_seed(seed)
    if ball_radius is not None:
        d = torch.randn((P, 3), generator=g)
        d = d / d.norm(dim=1, keepdim=True)
        r = ball_radius * torch.rand((P, 1), generator=g) ** (1.0 / 3.0)
        means = d * r
    else:
        assert cam is not None
        tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
        z = z_range[0] + (z_range[1] - z_range[0]) * torch.rand((P,), generator=g)
        x = (2 * torch.rand((P,), generator=g) - 1) * tx * z
        y = (2 * torch.rand((P,), generator=g) - 1) * ty * z
        pc = torch.stack([x, y, z], 1)
        # camera -> world with the camera's world_view_transform (row-vector convention)
        wvt_inv = cam.world_view_transform.double().inverse()
        ph = torch.cat([pc.double(), torch.ones((P, 1), dtype=torch.float64)], 1) @ wvt_inv
        means = ph[:, :3].float()
    lo, hi = math.log(scale_range[0]), math.log(scale_range[1])
    scales = torch.exp(lo + (hi - lo) * torch.rand((P, 3), generator=g))
    q = torch.randn((P, 4), generator=g)
    rots = torch.nn.functional.normalize(q)
    opac = torch.sigmoid(torch.randn((P, 1), generator=g))
    K = (sh_degree + 1) ** 2
    f_dc = ((torch.rand((P, 1, 3), generator=g) - 0.5) / SH_C0)
    f_rest = 0.05 * torch.randn((P, K - 1, 3), generator=g)
    shs = torch.cat([f_dc, f_rest], 1).contiguous()
    return GaussianScene(means.contiguous(), opac, scales, rots, shs, sh_degree)


def concat_scenes(*scenes: GaussianScene) -> GaussianScene:
    """Concatenate scenes of one SH degree (e.g. a skysphere-like mix of tiny and huge splats)."""
    cat = lambda f: torch.cat([getattr(s, f) for s in scenes], 0).contiguous()  # noqa: E731
    return GaussianScene(cat("means3D"), cat("opacities"), cat("scales"), cat("rotations"), cat("shs"),
                         scenes[0].sh_degree)


def raster_settings_for(cam: MiniCamera, sh_degree, bg=None, scale_modifier=1.0, debug=False, device="cuda"):
    """The settings the reference adapter builds (gaussian_renderer/__init__.py:33-49)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings

    if bg is None:
        bg = torch.zeros(3, dtype=torch.float32, device=device)
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg,
        scale_modifier=scale_modifier, viewmatrix=cam.world_view_transform.to(device),
        projmatrix=cam.full_proj_transform.to(device), sh_degree=sh_degree,
        campos=cam.camera_center.to(device), prefiltered=False, debug=debug)


def dl_dimage(H, W, seed=1, scale=1e-3):
    g = torch.Generator().manual_seed(seed)
    return scale * torch.randn((3, H, W), generator=g)
