"""bench.py's roofline bookkeeping (CPU): the committed PMC counters (profiles/<tag>_traffic.json, one
64-view launch of the default workload) are attributed per launch scaled by the views a rank launches,
and omitted for workloads they were not measured on."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(*extra):
    old = sys.argv
    sys.argv = ["bench.py", *extra]
    try:
        return bench.parse()
    finally:
        sys.argv = old


PHASES = {"render_fwd": (3.2, 1), "render_bwd": (7.1, 1), "binning": (4.4, 1), "preprocess": (2.0, 1)}


def test_counters_scale_with_views_per_launch():
    a = _args()
    full = bench.roofline_fields(a, PHASES, [6.6e6] * 64, [4.95e6] * 64, 1024, 1024)
    half = bench.roofline_fields(a, PHASES, [6.6e6] * 32, [4.95e6] * 32, 1024, 1024)
    t64, t32 = full["roofline"]["traffic"], half["roofline"]["traffic"]
    assert full["roofline"]["kernel"] == "k_render_bwd" and t64 is not None and t64 > 0
    assert abs(t32 - t64 / 2) <= 1
    v64, v32 = full["roofline"]["valu"]["insts_per_launch"], half["roofline"]["valu"]["insts_per_launch"]
    assert abs(v32 - v64 / 2) <= 1
    # instructions per pair do not depend on the split
    assert full["roofline"]["valu"]["valu_insts_per_64_pairs"] == half["roofline"]["valu"]["valu_insts_per_64_pairs"]


def test_roofline_is_the_slower_blend_not_the_dominant_phase():
    a = _args()
    ph = dict(PHASES, binning=(50.0, 1))
    r = bench.roofline_fields(a, ph, [6.6e6] * 64, [4.95e6] * 64, 1024, 1024)
    assert r["dominant_kernel"] == "binning" and r["roofline"]["kernel"] == "k_render_bwd"


def test_no_counters_for_unprofiled_workloads():
    for extra in (["--workload", "sugar"], ["--epilogue", "shading"], ["--res", "512"]):
        r = bench.roofline_fields(_args(*extra), PHASES, [1e6] * 64, [8e5] * 64, 512, 512)
        assert r["roofline"]["traffic"] is None and "valu" not in r["roofline"], extra
        assert "counters_note" in r


def test_c5_line_reads_its_own_counters():
    """The C5 line (--workload sugar at its 800^2) takes the two-colour kernels' counters from
    profiles/r03d_sugar_traffic.json (hit-list backward, quadrant-wave two-colour forward)."""
    a = _args("--workload", "sugar", "--res", "800")
    r = bench.roofline_fields(a, PHASES, [2.7e6] * 64, [2.69e6] * 64, 800, 800)
    assert r["roofline"]["traffic"] is not None and r["roofline"]["traffic"] > 0
    assert r["roofline_fwd_blend"]["traffic"] is not None
    assert "counters_note" not in r and "barriers" in r["roofline"]["limiter"]
