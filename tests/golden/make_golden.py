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
"""
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


if __name__ == "__main__":
    sh_utils, gu, gfx = _import_ref()
    sh_vectors(sh_utils)
    cov_vectors(gu)
    camera_vectors(gfx)
    loss_vectors()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
