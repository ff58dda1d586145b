"""Fused SSIM / L1 (gs_loss, csrc/gs_loss.hip) against the reference loss
(/root/reference/utils/loss_utils.py via tests/golden/loss_golden.npz) and the fp64 CPU
restatement oracle/ssim_oracle.py.

Tolerances: the oracle is float64 and pinned to the reference's float32 outputs at 2e-6 (value)
and 1e-5 relative + 1e-5 x max (gradient); the HIP kernels compute in float32 with a separable
window, checked against the oracle at 2e-6 (value) and 1e-5 relative + 1e-5 x max (gradient)."""
import numpy as np
import pytest
import torch

from oracle import ssim_oracle

G = np.load(__file__.rsplit("/", 1)[0] + "/golden/loss_golden.npz")
CASES = ["chw", "bchw", "tiny"]


def _close(a, b, rtol=1e-5, frac=1e-5, name=""):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    tol = rtol * np.abs(b) + frac * max(np.abs(b).max(), 1e-30)
    assert (np.abs(a - b) <= tol).all(), f"{name}: max|d| {np.abs(a - b).max():.3e} max|ref| {np.abs(b).max():.3e}"


def test_window_matches_reference():
    np.testing.assert_array_equal(ssim_oracle.window1d().numpy(), G["window1d"])


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_golden(case):
    a = torch.tensor(G[f"{case}_img1"], requires_grad=True)
    b = torch.tensor(G[f"{case}_img2"])
    s = ssim_oracle.ssim(a, b)
    s.backward()
    assert abs(s.item() - float(G[f"{case}_ssim"])) < 2e-6
    _close(a.grad.numpy(), G[f"{case}_grad"], name="grad")
    assert abs(ssim_oracle.l1_loss(a, b).item() - float(G[f"{case}_l1"])) < 1e-6
    if f"{case}_ssim_per_image" in G.files:
        a3 = torch.tensor(G[f"{case}_img1"], requires_grad=True)
        s3 = ssim_oracle.ssim(a3, b, size_average=False)
        s3.sum().backward()
        np.testing.assert_allclose(s3.detach().numpy(), G[f"{case}_ssim_per_image"], atol=2e-6)
        _close(a3.grad.numpy(), G[f"{case}_grad_per_image_sum"], name="grad per image")


def test_gs_loss_window_and_cpu_refusal():
    import gs_loss

    np.testing.assert_array_equal(np.array(list(gs_loss._WIN), np.float32), G["window1d"])
    with pytest.raises(RuntimeError, match="no CPU path"):
        gs_loss.ssim(torch.rand(3, 8, 8), torch.rand(3, 8, 8))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_ssim_matches_reference_golden(case, device):
    import gs_loss

    a = torch.tensor(G[f"{case}_img1"], device=device, requires_grad=True)
    b = torch.tensor(G[f"{case}_img2"], device=device)
    s = gs_loss.ssim(a, b)
    s.backward()
    assert abs(s.item() - float(G[f"{case}_ssim"])) < 2e-6
    _close(a.grad.cpu().numpy(), G[f"{case}_grad"], name="grad")
    if f"{case}_ssim_per_image" in G.files:
        a3 = torch.tensor(G[f"{case}_img1"], device=device, requires_grad=True)
        s3 = gs_loss.ssim(a3, b, size_average=False)
        s3.sum().backward()
        np.testing.assert_allclose(s3.detach().cpu().numpy(), G[f"{case}_ssim_per_image"], atol=2e-6)
        _close(a3.grad.cpu().numpy(), G[f"{case}_grad_per_image_sum"], name="grad per image")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 270, 480), (2, 3, 64, 80), (3, 1080, 1920), (3, 5, 7), (3, 1, 40)])
def test_gpu_ssim_matches_oracle(shape, device):
    """Including the full 1080p frame of train.py (16x16 tiles, ragged borders)."""
    import gs_loss

    g = torch.Generator().manual_seed(5)
    a0 = torch.rand(shape, generator=g)
    b0 = (a0 + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
    ref_a = a0.clone().requires_grad_(True)
    ref = ssim_oracle.ssim(ref_a, b0)
    ref.backward()
    a = a0.to(device).requires_grad_(True)
    s = gs_loss.ssim(a, b0.to(device))
    (2.5 * s).backward()
    assert abs(s.item() - ref.item()) < 2e-6
    _close(a.grad.cpu().numpy() / 2.5, ref_a.grad.numpy(), name="grad")
    l1 = gs_loss.l1_loss(a, b0.to(device))
    assert abs(l1.item() - ssim_oracle.l1_loss(a0, b0).item()) < 1e-6


def test_photometric_loss_cpu_refusal():
    import gs_loss

    with pytest.raises(RuntimeError, match="no CPU path"):
        gs_loss.photometric_loss(torch.rand(3, 8, 8), torch.rand(3, 8, 8))


def _oracle_photometric(a0, b0, lam):
    ref_a = a0.clone().requires_grad_(True)
    l1 = ssim_oracle.l1_loss(ref_a, b0)
    loss = (1.0 - lam) * l1 + lam * (1.0 - ssim_oracle.ssim(ref_a, b0))
    loss.backward()
    return loss.item(), l1.item(), ref_a.grad.numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("shape,lam", [((3, 270, 480), 0.2), ((2, 3, 64, 80), 0.2), ((3, 1080, 1920), 0.2),
                                       ((3, 37, 53), 0.7), ((1, 16, 16), 0.0), ((3, 20, 21), 1.0),
                                       ((3, 5, 7), 0.2), ((3, 1, 40), 0.2), ((2, 33, 1), 0.5)])
def test_gpu_photometric_loss_matches_oracle(shape, lam, device):
    """train.py:91-92 fused (gs_loss.photometric_loss) against the fp64 oracle of the same expression:
    value within 2e-6, gradient within 1e-5 relative + 1e-5 x max; pixels with image == gt (L1
    subgradient 0, as torch's abs backward) included."""
    import gs_loss

    g = torch.Generator().manual_seed(11)
    a0 = torch.rand(shape, generator=g)
    b0 = (a0 + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
    eq = torch.rand(shape, generator=g) < 0.05
    b0 = torch.where(eq, a0, b0)
    ref_loss, ref_l1, ref_grad = _oracle_photometric(a0, b0, lam)
    a = a0.to(device).requires_grad_(True)
    loss, l1 = gs_loss.photometric_loss(a, b0.to(device), lam)
    assert not l1.requires_grad and loss.requires_grad and loss.dim() == 0
    (3.0 * loss).backward()
    assert abs(loss.item() - ref_loss) < 2e-6 and abs(l1.item() - ref_l1) < 1e-6
    _close(a.grad.cpu().numpy() / 3.0, ref_grad, name="grad")


@pytest.mark.gpu
def test_gpu_photometric_loss_matches_separate_terms(device):
    """The fused expression against gs_loss.l1_loss + gs_loss.ssim composed by torch as train.py does."""
    import gs_loss

    g = torch.Generator().manual_seed(12)
    a0 = torch.rand((3, 130, 170), generator=g).to(device)
    b0 = torch.rand((3, 130, 170), generator=g).to(device)
    a1 = a0.clone().requires_grad_(True)
    Ll1 = gs_loss.l1_loss(a1, b0)
    loss1 = 0.8 * Ll1 + 0.2 * (1.0 - gs_loss.ssim(a1, b0))
    loss1.backward()
    a2 = a0.clone().requires_grad_(True)
    loss2, Ll2 = gs_loss.photometric_loss(a2, b0, 0.2)
    loss2.backward()
    assert abs(loss1.item() - loss2.item()) <= 1e-6 * abs(loss1.item())
    assert abs(Ll1.item() - Ll2.item()) <= 1e-6 * abs(Ll1.item())
    _close(a2.grad.cpu().numpy(), a1.grad.cpu().numpy(), rtol=1e-5, frac=1e-6, name="grad")
