"""Host-side API of the drop-in package (no GPU): names, field order, the reference's exceptions, and that
the product path refuses to run on the CPU instead of silently falling back."""
import pytest
import torch

import diff_gaussian_rasterization as dgr
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C


def _settings():
    return GaussianRasterizationSettings(image_height=32, image_width=32, tanfovx=0.5, tanfovy=0.5,
                                         bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4),
                                         projmatrix=torch.eye(4), sh_degree=0, campos=torch.zeros(3),
                                         prefiltered=False, debug=False)


def test_public_names():
    for name in ("GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians"):
        assert hasattr(dgr, name)
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug")


def test_exactly_one_of_sh_or_colors():
    r = GaussianRasterizer(_settings())
    x = torch.zeros(4, 3)
    with pytest.raises(Exception, match="SHs or precomputed colors"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), scales=x, rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="SHs or precomputed colors"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), colors_precomp=x,
          scales=x, rotations=torch.zeros(4, 4))


def test_exactly_one_of_scale_rotation_or_cov():
    r = GaussianRasterizer(_settings())
    x = torch.zeros(4, 3)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x,
          rotations=torch.zeros(4, 4), cov3D_precomp=torch.zeros(4, 6))


def test_no_cpu_fallback():
    r = GaussianRasterizer(_settings())
    x = torch.zeros(4, 3)
    with pytest.raises(_C.GSRError, match="GPU"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x,
          rotations=torch.zeros(4, 4))


def test_means_shape_check():
    with pytest.raises(_C.GSRError, match=r"num_points, 3"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(4, 2), None, None, None, None, 1.0, None, None, None,
                               0.5, 0.5, 8, 8, None, 0, None, False, False)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError, match="HIP library not found"):
        _C.load_library(str(tmp_path / "nope.so"))
