"""The per-tile list bounds by search (csrc/gsr_binning.hip k_tile_bounds), restated
step for step on the CPU: a fixed-step lower bound (trip count floor(log2 K) + 1, the same for every thread of a
view) over a list sorted by tile id, written as tile t's start and tile t - 1's end.  Checked against numpy's
searchsorted and against the scan's definition (first / last position of each tile id; empty tiles empty) on
ragged, empty, single-tile and packed-key lists.  The GPU kernel itself is held bitwise to the streaming scan by
tests/test_gpu_parity.py::test_forward_kernels_bitwise[*-tile_ranges]."""
import numpy as np
import pytest


def lower_bound_fixed_step(keys, K, t, gbits, tmask):
    """k_tile_bounds' search for one boundary t (the kernel's loop, integer for integer)."""
    lo = 0
    step = 0 if K == 0 else 1 << (K.bit_length() - 1)
    while step > 0:
        m = lo + step
        if m <= K and ((int(keys[m - 1]) >> gbits) & tmask) < t:
            lo = m
        step >>= 1
    return lo


def tile_bounds(keys, K, n_tiles, gbits, tmask):
    ranges = np.zeros((n_tiles, 2), np.int64)
    for t in range(n_tiles + 1):
        b = lower_bound_fixed_step(keys, K, t, gbits, tmask)
        if t < n_tiles:
            ranges[t, 0] = b
        if t > 0:
            ranges[t - 1, 1] = b
    return ranges


def scan_ranges(tiles, n_tiles):
    """The streaming definition (k_tile_ranges / identifyTileRanges): [first, last + 1) of each tile id, (0, 0) for
    tiles without instances."""
    r = np.zeros((n_tiles, 2), np.int64)
    for p, t in enumerate(tiles):
        if p == 0 or tiles[p - 1] != t:
            r[t, 0] = p
        if p == len(tiles) - 1 or tiles[p + 1] != t:
            r[t, 1] = p + 1
    return r


def same_lists(a, b):
    """Equal as lists: the same (start, end) for non-empty tiles, empty for the others (the search puts an empty
    tile's range at its neighbour's bound, the scan at (0, 0))."""
    na, nb = a[:, 1] - a[:, 0], b[:, 1] - b[:, 0]
    if not np.array_equal(na, nb):
        return False
    nz = na > 0
    return np.array_equal(a[nz], b[nz]) and (na >= 0).all()


@pytest.mark.parametrize("case", ["random", "empty", "one", "single_tile", "ragged_edges", "packed"])
def test_tile_bounds_match_scan(case):
    rng = np.random.default_rng({"random": 1, "empty": 2, "one": 3, "single_tile": 4, "ragged_edges": 5,
                                 "packed": 6}[case])
    n_tiles, gbits, tmask = 64, 0, 0xFFF
    if case == "random":
        tiles = np.sort(rng.integers(0, n_tiles, 3000))
    elif case == "empty":
        tiles = np.zeros(0, np.int64)
    elif case == "one":
        tiles = np.array([17])
    elif case == "single_tile":
        tiles = np.full(777, 5)
    elif case == "ragged_edges":  # first and last tiles used, long empty stretches between
        tiles = np.sort(np.concatenate([np.zeros(9, np.int64), np.full(4, n_tiles - 1), rng.integers(30, 33, 50)]))
    else:  # packed (tile << gbits | Gaussian) keys with 4-bit quadrant masks above the tile field
        gbits, tmask = 20, 0xFF
        tiles = np.sort(rng.integers(0, n_tiles, 2500))
    K = len(tiles)
    keys = tiles.astype(np.int64) << gbits
    if case == "packed":
        keys = keys | rng.integers(0, 1 << gbits, K) | (rng.integers(0, 16, K) << 28)
    got = tile_bounds(keys, K, n_tiles, gbits, tmask)
    assert same_lists(got, scan_ranges(tiles, n_tiles))
    # every start is numpy's left insertion point of the tile id
    assert np.array_equal(got[:, 0], np.searchsorted(tiles, np.arange(n_tiles), side="left"))
    # the live count bounds the search: positions past K (stale keys of the buffer) are never read
    if K > 0:
        junk = np.concatenate([keys, np.zeros(100, np.int64)])
        assert np.array_equal(tile_bounds(junk, K, n_tiles, gbits, tmask), got)
