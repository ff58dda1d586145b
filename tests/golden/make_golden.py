"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE's own Python code.

Run only in the build container, where /root/reference exists:
    python tests/golden/make_golden.py
The reference never travels to the GPU box; only the .npz outputs are committed.

Reference functions exercised (all on CPU):
  - utils/sh_utils.py:57-100           eval_sh (forward + autograd backward), deg 0..3
  - utils/general_utils.py:78-110      build_rotation / build_scaling_rotation / strip_symmetric, via
                                       a shim that drops their hard-coded device="cuda" (:65,83,102)
  - scene/gaussian_model.py:27-31      build_covariance_from_scaling_rotation (restated 3 lines: the
                                       module itself needs plyfile/simple_knn, absent here)
  - utils/graphics_utils.py:38-71      getWorld2View2, getProjectionMatrix
  - gaussian_renderer/__init__.py:73-78  convert_SHs_python colour path (+0.5, clamp_min 0)
  - utils/loss_utils.py:17-60          l1_loss, gaussian / create_window, ssim (+ autograd grads)
  - scene/gaussian_model.py:258-403    GaussianModel.densify_and_prune with its optimizer surgery, run
                                       on CPU: the module is loaded with empty stand-ins for the two
                                       imports it does not use on this path (plyfile, simple_knn._C) and
                                       the same device="cuda"-dropping torch proxy
  - gaussian_renderer/__init__.py:18-100  render() with the reference's own Camera (scene/cameras.py:
                                       17-57; its .cuda() calls made no-ops) and GaussianModel getters
                                       (:95-118); a recording stand-in for diff_gaussian_rasterization
                                       captures the settings and inputs it builds (render_golden.npz)
"""
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_ref():
    sys.path.insert(0, REF)
    import utils.sh_utils as sh_utils  # noqa
    import utils.general_utils as gu  # noqa
    import utils.graphics_utils as gfx  # noqa

    class _TorchCPU(types.ModuleType):
        """torch proxy whose zeros() ignores device= (the reference hard-codes cuda)."""

        def __getattr__(self, k):
            return getattr(torch, k)

        @staticmethod
        def zeros(*a, **kw):
            kw.pop("device", None)
            return torch.zeros(*a, **kw)

    gu.torch = _TorchCPU("torch")
    return sh_utils, gu, gfx


def sh_vectors(sh_utils):
    g = torch.Generator().manual_seed(1234)
    out = {}
    N = 256
    for deg in range(4):
        K = (deg + 1) ** 2
        sh = (0.5 * torch.randn((N, 16, 3), generator=g)).requires_grad_(True)   # [P, K, 3] like get_features
        d = torch.randn((N, 3), generator=g)
        d = (d / d.norm(dim=1, keepdim=True)).requires_grad_(True)
        shs_view = sh.transpose(1, 2)  # [P, 3, K]   (gaussian_renderer/__init__.py:74)
        rgb = sh_utils.eval_sh(deg, shs_view, d)
        colors = torch.clamp_min(rgb + 0.5, 0.0)
        w = torch.randn((N, 3), generator=g)
        (colors * w).sum().backward()
        out[f"deg{deg}_sh"] = sh.detach().numpy()
        out[f"deg{deg}_dirs"] = d.detach().numpy()
        out[f"deg{deg}_rgb"] = colors.detach().numpy()
        out[f"deg{deg}_w"] = w.numpy()
        out[f"deg{deg}_dsh"] = sh.grad.numpy()
        out[f"deg{deg}_ddirs"] = d.grad.numpy() if d.grad is not None else np.zeros((N, 3), np.float32)
    np.savez_compressed(os.path.join(OUT, "sh_golden.npz"), **out)


def cov_vectors(gu):
    g = torch.Generator().manual_seed(99)
    N = 256
    scales = torch.exp(torch.empty((N, 3)).uniform_(np.log(0.005), np.log(0.3), generator=g)).requires_grad_(True)
    q = torch.randn((N, 4), generator=g)
    q = (q / q.norm(dim=1, keepdim=True)).requires_grad_(True)
    out = {}
    for mod in (1.0, 0.7):
        if scales.grad is not None:
            scales.grad = None
            q.grad = None
        L = gu.build_scaling_rotation(mod * scales, q)          # gaussian_model.py:28
        cov = gu.strip_symmetric(L @ L.transpose(1, 2))          # gaussian_model.py:29-30
        w = torch.randn((N, 6), generator=g)
        (cov * w).sum().backward()
        tag = f"mod{mod}"
        out[f"{tag}_cov"] = cov.detach().numpy()
        out[f"{tag}_w"] = w.numpy()
        out[f"{tag}_dscales"] = scales.grad.numpy().copy()
        out[f"{tag}_drot"] = q.grad.numpy().copy()
    out["scales"] = scales.detach().numpy()
    out["rotations"] = q.detach().numpy()
    np.savez_compressed(os.path.join(OUT, "cov_golden.npz"), **out)


def camera_vectors(gfx):
    out = {}
    cases = [(0.01, 100.0, 1.2, 0.8), (0.01, 100.0, np.deg2rad(60.0) * 1.5, np.deg2rad(60.0)), (0.1, 50.0, 0.5, 0.9)]
    for i, (zn, zf, fx, fy) in enumerate(cases):
        out[f"proj{i}"] = gfx.getProjectionMatrix(znear=zn, zfar=zf, fovX=fx, fovY=fy).numpy()
        out[f"proj{i}_args"] = np.array([zn, zf, fx, fy])
    rng = np.random.default_rng(7)
    for i in range(3):
        A = rng.normal(size=(3, 3))
        Q, _ = np.linalg.qr(A)
        if np.linalg.det(Q) < 0:
            Q[:, 0] *= -1
        T = rng.normal(size=3)
        out[f"w2v{i}_R"] = Q
        out[f"w2v{i}_T"] = T
        out[f"w2v{i}"] = gfx.getWorld2View2(Q, T)
    out["focal2fov"] = np.array([gfx.focal2fov(1000.0, 1920), gfx.focal2fov(500.0, 800)])
    np.savez_compressed(os.path.join(OUT, "camera_golden.npz"), **out)


def loss_vectors():
    import utils.loss_utils as lu  # noqa

    g = torch.Generator().manual_seed(77)
    out = {"window1d": lu.gaussian(11, 1.5).numpy()}
    cases = {"chw": (3, 37, 45), "bchw": (2, 3, 20, 27), "tiny": (1, 7, 9)}
    for name, shape in cases.items():
        a = torch.rand(shape, generator=g)
        b = (a + 0.15 * torch.randn(shape, generator=g)).clamp(0, 1)
        a = a.requires_grad_(True)
        s = lu.ssim(a, b)
        s.backward()
        out[f"{name}_img1"] = a.detach().numpy()
        out[f"{name}_img2"] = b.numpy()
        out[f"{name}_ssim"] = np.array(s.item(), np.float64)
        out[f"{name}_grad"] = a.grad.numpy()
        a2 = a.detach().clone().requires_grad_(True)
        l1 = lu.l1_loss(a2, b)
        l1.backward()
        out[f"{name}_l1"] = np.array(l1.item(), np.float64)
        out[f"{name}_l1grad"] = a2.grad.numpy()
        if len(shape) == 4:  # size_average=False: per-image SSIM
            a3 = a.detach().clone().requires_grad_(True)
            s3 = lu.ssim(a3, b, size_average=False)
            s3.sum().backward()
            out[f"{name}_ssim_per_image"] = s3.detach().numpy()
            out[f"{name}_grad_per_image_sum"] = a3.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "loss_golden.npz"), **out)


def _ref_gaussian_model():
    """scene/gaussian_model.py imported on CPU (its plyfile / simple_knn imports are unused here)."""
    for name, attrs in (("plyfile", ("PlyData", "PlyElement")), ("simple_knn", ()), ("simple_knn._C", ("distCUDA2",))):
        if name not in sys.modules:
            m = types.ModuleType(name)
            for a in attrs:
                setattr(m, a, None)
            sys.modules[name] = m
    import scene.gaussian_model as gm  # noqa

    gm.torch = _TORCH_CPU
    return gm


class _TorchCPUProxy(types.ModuleType):
    """torch proxy whose zeros() ignores device= (the reference hard-codes cuda)."""

    def __getattr__(self, k):
        return getattr(torch, k)

    @staticmethod
    def zeros(*a, **kw):
        kw.pop("device", None)
        return torch.zeros(*a, **kw)


_TORCH_CPU = _TorchCPUProxy("torch")

DENSIFY_LRS = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3]
DENSIFY_NAMES = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]


def densify_inputs(P, seed):
    """Parameters / stats that exercise clone, split (kept and pruned children), NaN grads, opacity
    and world-size pruning with percent_dense 0.01, extent 2 (pd_extent 0.02, big 0.2), thr 2e-4."""
    g = torch.Generator().manual_seed(seed)
    d = {
        "xyz": torch.randn((P, 3), generator=g),
        "f_dc": torch.randn((P, 1, 3), generator=g),
        "f_rest": torch.randn((P, 15, 3), generator=g) * 0.1,
        "opacity": torch.randn((P, 1), generator=g) * 3.0,
        "scaling": math.log(0.003) + torch.rand((P, 3), generator=g) * (math.log(0.5) - math.log(0.003)),
        "rotation": torch.randn((P, 4), generator=g),
    }
    denom = torch.randint(0, 6, (P, 1), generator=g).float()
    accum = torch.rand((P, 1), generator=g) * 4e-4 * denom
    accum[denom == 0] = 0.0
    radii = torch.randint(0, 30, (P,), generator=g).float()
    grads = {k: torch.randn(v.shape, generator=g) for k, v in d.items()}
    return d, accum, denom, radii, grads


def densify_vectors(gm_mod):
    out = {}
    for case, (P, seed, screen) in {"a": (400, 11, 20), "b": (300, 12, None)}.items():
        d, accum, denom, radii, grads = densify_inputs(P, seed)
        m = gm_mod.GaussianModel(3)
        for n, attr in zip(DENSIFY_NAMES, ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling",
                                           "_rotation")):
            setattr(m, attr, torch.nn.Parameter(d[n].clone().requires_grad_(True)))
        m.percent_dense = 0.01
        groups = [{"params": [getattr(m, a)], "lr": lr, "name": n} for n, a, lr in
                  zip(DENSIFY_NAMES, ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"),
                      DENSIFY_LRS)]
        m.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        for _ in range(2):  # non-trivial Adam moments
            for grp in m.optimizer.param_groups:
                grp["params"][0].grad = grads[grp["name"]].clone()
            m.optimizer.step()
        for grp in m.optimizer.param_groups:
            n = grp["name"]
            out[f"{case}_in_{n}"] = grp["params"][0].detach().numpy().copy()
            st = m.optimizer.state[grp["params"][0]]
            out[f"{case}_in_{n}_exp_avg"] = st["exp_avg"].numpy().copy()
            out[f"{case}_in_{n}_exp_avg_sq"] = st["exp_avg_sq"].numpy().copy()
            m.optimizer.state[grp["params"][0]] = st
        m.xyz_gradient_accum, m.denom, m.max_radii2D = accum.clone(), denom.clone(), radii.clone()
        out[f"{case}_in_accum"], out[f"{case}_in_denom"], out[f"{case}_in_max_radii2D"] = (
            accum.numpy(), denom.numpy(), radii.numpy())
        out[f"{case}_args"] = np.array([2e-4, 0.005, 2.0, -1.0 if screen is None else screen, seed], np.float64)
        torch.manual_seed(seed)
        m.densify_and_prune(2e-4, 0.005, 2.0, screen)
        for grp in m.optimizer.param_groups:
            n = grp["name"]
            out[f"{case}_out_{n}"] = grp["params"][0].detach().numpy()
            st = m.optimizer.state[grp["params"][0]]
            out[f"{case}_out_{n}_exp_avg"] = st["exp_avg"].numpy()
            out[f"{case}_out_{n}_exp_avg_sq"] = st["exp_avg_sq"].numpy()
            out[f"{case}_out_{n}_step"] = np.array(float(st["step"]))
        out[f"{case}_out_sizes"] = np.array([m.xyz_gradient_accum.shape[0], m.denom.shape[0], m.max_radii2D.shape[0]])
    np.savez_compressed(os.path.join(OUT, "densify_golden.npz"), **out)


# render() adapter cases: (W, H, fovy_deg, camera position, target or None for R=I/T=0, sh degree
# active/max, scale_modifier, compute_cov3D_python, convert_SHs_python)
RENDER_CASES = {
    "c1": (256, 256, 60.0, None, None, 0, 0, 1.0, False, False),
    "c2": (800, 800, 60.0, None, None, 3, 3, 1.0, False, False),
    "c3": (1920, 1080, 60.0, None, None, 3, 3, 1.0, False, False),
    "c4v3": (1920, 1080, 60.0, (6.0 * math.cos(2 * math.pi * 3 / 8), 0.0, 6.0 * math.sin(2 * math.pi * 3 / 8)),
             (0.0, 0.0, 0.0), 3, 3, 1.0, False, False),
    "ring_py": (96, 64, 50.0, (1.5, -0.4, -3.0), (0.1, 0.2, 0.3), 1, 3, 0.7, True, True),
}


def _look_at_rt(position, target, up=(0.0, -1.0, 0.0)):
    """(R, T) in the reference loaders' storage convention (R = W2C^T, T = W2C translation) for an
    OpenCV-axes camera at `position` looking at `target` (the synthetic C4 ring)."""
    c = np.asarray(position, np.float64)
    f = np.asarray(target, np.float64) - c
    f /= np.linalg.norm(f)
    r = np.cross(f, np.asarray(up, np.float64))
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    w2c = np.stack([r, d, f], axis=0)
    return w2c.T, -w2c @ c


def render_vectors():
    """gaussian_renderer/__init__.py:18-100 driven with the reference's own Camera
    (scene/cameras.py:17-57, its two .cuda() calls made no-ops on CPU) and GaussianModel
    (getters :95-118), with a recording stand-in for diff_gaussian_rasterization: captures the exact
    GaussianRasterizationSettings and rasterizer inputs render() hands over."""
    rec = {}

    class Settings(tuple):
        _fields = ("image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix",
                   "projmatrix", "sh_degree", "campos", "prefiltered", "debug")

        def __new__(cls, **kw):
            rec["settings"] = kw
            return tuple.__new__(cls, [kw[f] for f in cls._fields])

    class Rasterizer:
        def __init__(self, raster_settings):
            self.s = raster_settings

        def __call__(self, **kw):
            rec["inputs"] = kw
            P = kw["means3D"].shape[0]
            return torch.zeros((3, self.s[0], self.s[1])), torch.zeros(P, dtype=torch.int32)

    stub = types.ModuleType("diff_gaussian_rasterization")
    stub.GaussianRasterizationSettings, stub.GaussianRasterizer = Settings, Rasterizer
    saved = sys.modules.get("diff_gaussian_rasterization")
    sys.modules["diff_gaussian_rasterization"] = stub
    gm = _ref_gaussian_model()
    sys.modules.pop("gaussian_renderer", None)
    import gaussian_renderer as gr  # noqa
    import scene.cameras as cams  # noqa
    if saved is not None:
        sys.modules["diff_gaussian_rasterization"] = saved

    class _RendererTorch(_TorchCPUProxy):  # render() allocates its carrier with device="cuda"
        @staticmethod
        def zeros_like(*a, **kw):
            kw.pop("device", None)
            return torch.zeros_like(*a, **kw)

    gr.torch = _RendererTorch("torch")
    out = {}
    cuda = torch.Tensor.cuda
    for name, (W, H, fovy_deg, pos, tgt, deg_act, deg_max, mod, cov_py, sh_py) in RENDER_CASES.items():
        if pos is None:
            R, T = np.eye(3), np.zeros(3)
        else:
            R, T = _look_at_rt(pos, tgt)
        fovy = math.radians(fovy_deg)
        fovx = 2.0 * math.atan(math.tan(fovy / 2.0) * W / H)
        torch.Tensor.cuda = lambda self, *a, **k: self
        try:
            cam = cams.Camera(colmap_id=0, R=R, T=T, FoVx=fovx, FoVy=fovy, image=torch.zeros((3, H, W)),
                              gt_alpha_mask=None, image_name=name, uid=0, data_device="cpu")
        finally:
            torch.Tensor.cuda = cuda
        g = torch.Generator().manual_seed(len(name) * 31 + W)
        P = 64
        m = gm.GaussianModel(deg_max)
        m.active_sh_degree = deg_act
        K = (deg_max + 1) ** 2
        m._xyz = torch.nn.Parameter(torch.randn((P, 3), generator=g) + torch.tensor([0.0, 0.0, 4.0]))
        m._features_dc = torch.nn.Parameter(torch.randn((P, 1, 3), generator=g))
        m._features_rest = torch.nn.Parameter(0.1 * torch.randn((P, K - 1, 3), generator=g))
        m._opacity = torch.nn.Parameter(torch.randn((P, 1), generator=g))
        m._scaling = torch.nn.Parameter(math.log(0.05) + torch.randn((P, 3), generator=g))
        m._rotation = torch.nn.Parameter(torch.randn((P, 4), generator=g))
        pipe = types.SimpleNamespace(debug=False, compute_cov3D_python=cov_py, convert_SHs_python=sh_py)
        bg = torch.tensor([0.0, 0.5, 1.0]) if sh_py else torch.zeros(3)
        rec.clear()
        gr.render(cam, m, pipe, bg, scaling_modifier=mod)
        s, x = rec["settings"], rec["inputs"]
        out[f"{name}_case"] = np.array([W, H, fovy_deg, deg_act, deg_max, mod, cov_py, sh_py], np.float64)
        out[f"{name}_R"], out[f"{name}_T"] = R, T
        out[f"{name}_fov"] = np.array([fovx, fovy], np.float64)
        out[f"{name}_hw"] = np.array([s["image_height"], s["image_width"]], np.int64)
        out[f"{name}_tanfov"] = np.array([s["tanfovx"], s["tanfovy"]], np.float64)
        for k in ("bg", "viewmatrix", "projmatrix", "campos"):
            out[f"{name}_{k}"] = s[k].detach().numpy()
        out[f"{name}_scalars"] = np.array([s["scale_modifier"], s["sh_degree"], s["prefiltered"], s["debug"]],
                                          np.float64)
        for p in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
            out[f"{name}_param{p}"] = getattr(m, p).detach().numpy()
        for k, v in x.items():
            if v is not None:
                out[f"{name}_in_{k}"] = v.detach().numpy()
    np.savez_compressed(os.path.join(OUT, "render_golden.npz"), **out)


if __name__ == "__main__":
    sh_utils, gu, gfx = _import_ref()
    sh_vectors(sh_utils)
    cov_vectors(gu)
    camera_vectors(gfx)
    loss_vectors()
    densify_vectors(_ref_gaussian_model())
    render_vectors()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
