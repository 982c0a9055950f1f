"""The view-segmented stable radix sort (csrc/gsr_sort.hip; every sort of the library: depth, tile and Morton keys)
through its C-ABI entry gsr_sort_pairs, against numpy's stable sort (the scatter's per-wave running
counts are read by every lane and advanced by each digit's first lane — many equal digits per wave, ragged segment
tails, empty and one-item segments, full 4096-item blocks and bounded last blocks, keys-only and key/value, 4-, 6-
and 8-bit digits and the runtime-width path).  Bit-exact: integer work."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEGS = [0, 1, 63, 64, 4095, 4096, 4097, 12288, 20000 + 37, 0, 5]


def _sort(keys, vals, sizes, key_bits, max_bits):
    import torch

    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    n = (ctypes.c_int * len(sizes))(*sizes)
    k = torch.tensor(keys.view(np.int32), device="cuda")
    v = torch.tensor(vals.view(np.int32), device="cuda") if vals is not None else None
    wb = lib.gsr_sort_work_bytes(len(sizes), n)
    assert wb > 0
    work = torch.empty(wb, dtype=torch.uint8, device="cuda")
    rc = lib.gsr_sort_pairs(len(sizes), n, ctypes.c_void_p(k.data_ptr()),
                            ctypes.c_void_p(v.data_ptr()) if v is not None else None, key_bits, max_bits,
                            ctypes.c_void_p(work.data_ptr()), wb, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.gsr_last_error()
    torch.cuda.synchronize()
    return k.cpu().numpy().view(np.uint32), (v.cpu().numpy().view(np.uint32) if v is not None else None)


def _expect(keys, vals, sizes, key_bits):
    mask = np.uint32(0xFFFFFFFF) if key_bits == 32 else np.uint32((1 << key_bits) - 1)
    ek, ev, o = keys.copy(), (vals.copy() if vals is not None else None), 0
    for n in sizes:
        seg = keys[o:o + n]
        order = np.argsort(seg & mask, kind="stable")
        ek[o:o + n] = seg[order]
        if vals is not None:
            ev[o:o + n] = vals[o:o + n][order]
        o += n
    return ek, ev


@pytest.mark.parametrize("key_bits,max_bits", [(32, 8), (12, 6), (30, 8), (8, 4), (13, 5), (20, 7)])
@pytest.mark.parametrize("distinct", [3, 64, 1 << 20])
@pytest.mark.parametrize("with_vals", [True, False])
def test_sort_pairs_matches_stable_sort(key_bits, max_bits, distinct, with_vals):
    rng = np.random.default_rng(key_bits * 1000 + max_bits * 10 + distinct % 97)
    total = sum(SEGS)
    # few distinct keys: long runs of equal digits in every wave and round (the running-count path); high bits above
    # key_bits set at random (ignored by the sort, carried along)
    keys = rng.integers(0, distinct, size=total, dtype=np.uint64).astype(np.uint32)
    if key_bits < 32:
        keys = (keys & np.uint32((1 << key_bits) - 1)) | (rng.integers(0, 2, size=total, dtype=np.uint32)
                                                         << np.uint32(key_bits))
    vals = np.arange(total, dtype=np.uint32) if with_vals else None
    gk, gv = _sort(keys, vals, SEGS, key_bits, max_bits)
    ek, ev = _expect(keys, vals, SEGS, key_bits)
    np.testing.assert_array_equal(gk, ek)
    if with_vals:
        np.testing.assert_array_equal(gv, ev)  # stability: equal keys keep their input order


def test_sort_pairs_all_equal_and_descending():
    """One digit for a whole segment (every lane of every round a peer of every other), and reversed input."""
    sizes = [4096 * 3 + 17, 8191]
    keys = np.concatenate([np.full(sizes[0], 0xABCDEF12, np.uint32),
                           np.arange(sizes[1], 0, -1, dtype=np.uint32)])
    vals = np.arange(sum(sizes), dtype=np.uint32)
    gk, gv = _sort(keys, vals, sizes, 32, 8)
    ek, ev = _expect(keys, vals, sizes, 32)
    np.testing.assert_array_equal(gk, ek)
    np.testing.assert_array_equal(gv, ev)


def test_rank_mode_probe_selects_lds_atomics():
    """The scatter ranks equal digits with LDS atomic adds only after the once-per-process probe found the device
    servicing same-counter lanes in lane order (gsr_sort.hip k_lds_rank_probe); on MI355X it does, so the fast
    path is the one the other tests here check against numpy's stable sort."""
    from diff_gaussian_rasterization import _C

    assert _C.load_library().gsr_sort_rank_mode() == 1


def test_ballot_ranks_give_the_same_bits(tmp_path):
    """GSR_SORT_RANK=ballot (read once per process: a child process) sorts to the same bits as the default."""
    import os
    import subprocess
    import sys

    rng = np.random.default_rng(7)
    sizes = [4096 * 2 + 5, 777, 12288]
    keys = rng.integers(0, 64, size=sum(sizes), dtype=np.uint64).astype(np.uint32)
    vals = np.arange(sum(sizes), dtype=np.uint32)
    np.save(tmp_path / "k.npy", keys)
    np.save(tmp_path / "v.npy", vals)
    code = (
        "import sys, numpy as np; sys.path[:0] = [%r, %r]; import test_gpu_sort as t; from diff_gaussian_rasterization "
        "import _C; k = np.load(%r); v = np.load(%r); gk, gv = t._sort(k, v, %r, 32, 6); "
        "np.save(%r, gk); np.save(%r, gv); print(_C.load_library().gsr_sort_rank_mode())"
        % (os.path.dirname(os.path.abspath(__file__)),
           os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "threestudio-3dgs_amd"),
           str(tmp_path / "k.npy"), str(tmp_path / "v.npy"), sizes,
           str(tmp_path / "bk.npy"), str(tmp_path / "bv.npy")))
    env = dict(os.environ, GSR_SORT_RANK="ballot")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "0"  # the child ranked by ballot matching
    gk, gv = _sort(keys, vals, sizes, 32, 6)
    np.testing.assert_array_equal(gk, np.load(tmp_path / "bk.npy"))
    np.testing.assert_array_equal(gv, np.load(tmp_path / "bv.npy"))
