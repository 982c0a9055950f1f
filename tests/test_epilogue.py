"""Fused background composite (include/gsr.h gsr_composite_*) against the reference's torch epilogue
(renderer/diff_gaussian_rasterizer_background.py:129-132, 139): forward bit-identical, gradients of
color / alpha / background equal to torch autograd of the same expression."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _reference(color, alpha, bg_hwc):
    H, W = color.shape[-2:]
    return (color + (1 - alpha) * bg_hwc.reshape(-1, H, W, 3).permute(0, 3, 1, 2)).clamp(0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 64, 48), (5, 40, 36), (2, 30, 17)])
def test_composite_matches_torch(shape):
    from diff_gaussian_rasterization.composite import composite_background

    V, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(V * 1000 + H)
    # values straddling the clamp bounds, incl. exact 0 / 1 pre-clamp values
    color = (torch.rand((V, 3, H, W), generator=g, device="cuda") * 1.4 - 0.2)
    color[:, 0, 0, 0] = 0.0
    alpha = torch.rand((V, 1, H, W), generator=g, device="cuda")
    alpha[:, 0, 0, :3] = 1.0
    bg = torch.rand((V, H, W, 3), generator=g, device="cuda")
    up = torch.randn((V, 3, H, W), generator=g, device="cuda")
    leaves = [t.clone().requires_grad_(True) for t in (color, alpha, bg)]
    ref = _reference(*leaves)
    ref.backward(up)
    mine = [t.clone().requires_grad_(True) for t in (color, alpha, bg)]
    out = composite_background(*mine)
    out.backward(up)
    assert torch.equal(out, ref)
    for a, b in zip(mine, leaves):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.cpu().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_composite_single_view_and_constant_background():
    from diff_gaussian_rasterization.composite import composite_background

    H, W = 32, 24
    g = torch.Generator(device="cuda").manual_seed(3)
    color = torch.rand((3, H, W), generator=g, device="cuda").requires_grad_(True)
    alpha = torch.rand((1, H, W), generator=g, device="cuda").requires_grad_(True)
    bgc = torch.tensor([0.5, 0.25, 1.0], device="cuda")
    out = composite_background(color, alpha, bgc)
    ref = (color + (1 - alpha) * bgc[:, None, None]).clamp(0, 1)
    assert torch.equal(out, ref)
    up = torch.randn_like(ref)
    ga = torch.autograd.grad(out, (color, alpha), up)
    gr = torch.autograd.grad(ref, (color, alpha), up)
    for a, b in zip(ga, gr):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-7)


def test_composite_symbols_exported():
    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    assert hasattr(lib, "gsr_composite_forward") and hasattr(lib, "gsr_composite_backward")
