"""Host-side behaviour of the drop-in package that needs no GPU: the reference adapter's
argument contract (gaussian_renderer/__init__.py:36-93) and loud failure on CPU tensors."""
import pytest
import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C


def _settings(debug=False):
    eye = torch.eye(4)
    return GaussianRasterizationSettings(image_height=16, image_width=16, tanfovx=0.5, tanfovy=0.5,
                                         bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=eye, projmatrix=eye,
                                         sh_degree=0, campos=torch.zeros(3), prefiltered=False, debug=debug)


def test_settings_field_order_matches_reference_call_site():
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug")


def test_exactly_one_colour_source_required():
    r = GaussianRasterizer(_settings())
    m = torch.zeros((2, 3))
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=torch.ones(2, 1), scales=m, rotations=torch.zeros(2, 4))
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=torch.ones(2, 1), shs=torch.zeros(2, 1, 3), colors_precomp=m,
          scales=m, rotations=torch.zeros(2, 4))


def test_exactly_one_covariance_source_required():
    r = GaussianRasterizer(_settings())
    m = torch.zeros((2, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=m, means2D=m, opacities=torch.ones(2, 1), colors_precomp=m, scales=m)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=m, means2D=m, opacities=torch.ones(2, 1), colors_precomp=m, scales=m, rotations=torch.zeros(2, 4),
          cov3D_precomp=torch.zeros(2, 6))


def test_means3d_shape_error_message():
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros((2, 4)), torch.zeros((2, 3)), torch.ones(2), torch.Tensor([]),
                               torch.Tensor([]), 1.0, torch.Tensor([]), torch.eye(4), torch.eye(4), 0.5, 0.5, 16, 16,
                               torch.Tensor([]), 0, torch.zeros(3), False, False)


def test_cpu_tensors_fail_loudly_no_cpu_fallback():
    r = GaussianRasterizer(_settings())
    m = torch.zeros((2, 3))
    with pytest.raises(RuntimeError, match="no CPU rasterizer"):
        r(means3D=m, means2D=m, opacities=torch.ones(2, 1), colors_precomp=m, scales=m, rotations=torch.zeros(2, 4))


def test_simple_knn_cpu_fails_loudly():
    from simple_knn._C import distCUDA2

    with pytest.raises(RuntimeError, match="no CPU path"):
        distCUDA2(torch.zeros((5, 3)))


def test_binning_layout_count_inverts_buffer_bytes():
    """gs_binning_layout_count (ABI 14): the count a binning buffer of n bytes is laid out for -- the
    backward of a gs_forward_counted forward takes it in place of num_rendered."""
    lib = _C._lib
    for W, H in ((16, 16), (800, 800), (1920, 1080)):
        assert lib.gs_binning_layout_count(0, W, H) == 0
        for n in (1, 2, 63, 64, 65, 1000, 65_536, 1_234_567, 4_310_000, 40_000_000):
            b = lib.gs_binning_buffer_bytes(n, W, H)
            L = lib.gs_binning_layout_count(b, W, H)
            assert L >= n and lib.gs_binning_buffer_bytes(L, W, H) == b
            assert lib.gs_binning_buffer_bytes(L + 1, W, H) > b
            assert lib.gs_binning_layout_count(b - 1, W, H) < n


def test_torch_host_extension_loads():
    """The torch C++ host path is built in-tree and binds libgsrast.so's symbols (no GPU call)."""
    import os

    if os.environ.get("GSRAST_NO_EXT", "0") not in ("", "0"):
        pytest.skip("GSRAST_NO_EXT set")
    assert _C._EXT is not None, "diff_gaussian_rasterization/_gs_ext*.so missing: run setup_ext.py"
    for name in ("forward", "backward", "preprocess_views", "forward_prepared", "backward_render",
                 "backward_gaussians", "count_estimate", "set_count_estimate"):
        assert callable(getattr(_C._EXT, name))
    assert _C._EXT.count_estimate(7, 1000, 64, 48) == 0
    _C._EXT.set_count_estimate(7, 1000, 64, 48, 12345)
    assert _C._EXT.count_estimate(7, 1000, 64, 48) == 12345
    assert _C._EXT.count_estimate(7, 1001, 64, 48) == 0  # per shape
    _C._EXT.set_count_estimate(7, 1000, 64, 48, 0)
