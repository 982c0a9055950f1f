"""The gradient parity rule itself (tests/gsr_testutil.py check_grads / adjudicate), on CPU: the fp32 oracle
stands in for the GPU.  Unperturbed it passes; with a 1e-3 relative error injected into a few rows of one
tensor — far below what a count-only rule notices when the fp32 oracle itself misses the bar on many rows —
the row-wise rule |g - g64| <= max(bar, ROW_RATIO |g32 - g64|) must fail it."""
import numpy as np
import pytest

import gsr_testutil as gt
from gsr_testutil import gs, make_camera, run_oracle

KEYS = ["means3D", "means2D", "opacity", "sh", "scales", "rotations"]


@pytest.fixture(scope="module")
def ref():
    scene = gs.make_scene(3000, sh_degree=1, seed=9)
    cam = make_camera(96, 80)
    return run_oracle(scene, cam, [1.0, 1.0, 1.0], grads=gs.upstream_grads(80, 96, seed=3))


def _as_gpu(ref):
    return {"g_" + k: np.array(ref["b32"][k], copy=True) for k in KEYS}


def test_fp32_oracle_passes_its_own_rule(ref):
    st = gt.check_grads(_as_gpu(ref), ref, KEYS, "rule self-check")
    assert all(s["beyond_ratio"] == 0 and s["gpu_only_miss"] == 0 for s in st.values())


@pytest.mark.parametrize("key", ["means3D", "scales", "opacity"])
def test_injected_row_errors_fail(ref, key):
    gpu = _as_gpu(ref)
    g64 = np.asarray(ref["b64"][key], np.float64)
    mag = np.abs(g64).reshape(g64.shape[0], -1).max(1)
    rows = np.argsort(-mag)[:8]  # rows with real gradient
    g = gpu["g_" + key].reshape(g64.shape[0], -1)
    g[rows, 0] += np.float32(1e-3) * np.maximum(1.0, np.abs(g64.reshape(g64.shape[0], -1)[rows, 0])).astype(np.float32)
    with pytest.raises(AssertionError) as e:
        gt.check_grads(gpu, ref, [key], "perturbed")
    assert "'beyond_ratio': 8" in str(e.value)


def test_rowwise_binds_where_the_count_does_not():
    """An ill-conditioned tensor (the fp32 restatement misses the bar on 30 % of the rows, as at C5): the
    count-only rule accepts 8 corrupted rows; the row-wise rule rejects them.  A GPU whose errors track the
    fp32 oracle's (up to ROW_RATIO x) passes both."""
    rng = np.random.default_rng(0)
    n = 20000
    r64 = rng.standard_normal((n, 3)) * 50
    bar = gt.GRAD_TOL * np.maximum(1.0, np.abs(r64))
    noise = np.where(rng.random((n, 1)) < 0.3, 20.0, 0.2) * bar * rng.standard_normal((n, 3))
    r32 = r64 + noise
    faithful = r64 + noise * rng.uniform(0.5, 1.5, (n, 3))
    gt.adjudicate(faithful, r32, r64, bar, "synthetic", "faithful", rowwise=True)
    bad = faithful.copy()
    clean = np.nonzero(np.abs(noise).max(1) < 0.5 * bar.max(1))[0][:8]
    bad[clean, 1] += 1e-3 * np.maximum(1.0, np.abs(r64[clean, 1]))
    gt.adjudicate(bad, r32, r64, bar, "synthetic", "count only", rowwise=False)  # the count rule passes it
    with pytest.raises(AssertionError, match="max\\(bar"):
        gt.adjudicate(bad, r32, r64, bar, "synthetic", "row-wise", rowwise=True)
