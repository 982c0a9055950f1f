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
    assert full["roofline"]["kernel"] == bench.KERNELS["c3"][1] and t64 is not None and t64 > 0
    assert abs(t32 - t64 / 2) <= 1
    v64, v32 = full["roofline"]["valu"]["insts_per_launch"], half["roofline"]["valu"]["insts_per_launch"]
    assert abs(v32 - v64 / 2) <= 1
    # instructions per pair do not depend on the split
    assert full["roofline"]["valu"]["valu_insts_per_64_pairs"] == half["roofline"]["valu"]["valu_insts_per_64_pairs"]


def test_roofline_is_the_slower_blend_not_the_dominant_phase():
    a = _args()
    ph = dict(PHASES, binning=(50.0, 1))
    r = bench.roofline_fields(a, ph, [6.6e6] * 64, [4.95e6] * 64, 1024, 1024)
    assert r["dominant_kernel"] == "binning" and r["roofline"]["kernel"] == bench.KERNELS["c3"][1]


def test_no_counters_for_unprofiled_workloads():
    for extra in (["--workload", "sugar"], ["--epilogue", "shading"], ["--res", "512"]):
        r = bench.roofline_fields(_args(*extra), PHASES, [1e6] * 64, [8e5] * 64, 512, 512)
        assert r["roofline"]["traffic"] is None and "valu" not in r["roofline"], extra
        assert "counters_note" in r


def test_c5_line_reads_its_own_counters():
    """The C5 line (--workload sugar at its 800^2) takes the two-colour kernels' counters from its own traffic file
    (the tile-wave hit-list backward, the quadrant-wave two-colour forward)."""
    a = _args("--workload", "sugar", "--res", "800")
    r = bench.roofline_fields(a, PHASES, [2.7e6] * 64, [2.69e6] * 64, 800, 800)
    assert r["roofline"]["traffic"] is not None and r["roofline"]["traffic"] > 0
    assert r["roofline_fwd_blend"]["traffic"] is not None
    assert "counters_note" not in r and "not HBM" in r["roofline"]["limiter"]


def test_committed_counters_name_the_timed_kernels():
    """The default traffic files hold counters of exactly the kernels the bench times (bench.KERNELS), so a
    kernel renamed or replaced in the build cannot borrow another kernel's counters."""
    a = _args()
    for path, kind in ((a.traffic, "c3"), (a.traffic_sugar, "sugar")):
        for kernel in bench.KERNELS[kind]:
            assert bench.read_traffic(path, kernel) is not None, (path, kernel)
            assert bench.read_traffic(path, kernel, "valu_insts_per_launch") is not None, (path, kernel)


def test_fwd_counters_only_for_the_profiled_launch():
    """At 32 views per launch (a rank's share at N = 2) the forward is the quadrant-wave kernel, not the profiled
    tile-wave one: no forward counters; the backward's scale with the views."""
    r = bench.roofline_fields(_args(), PHASES, [6.6e6] * 32, [4.95e6] * 32, 1024, 1024)
    assert r["roofline_fwd_blend"]["traffic"] is None and r["roofline"]["traffic"] is not None


def test_stale_counter_file_gives_no_fields(tmp_path):
    import json

    f = tmp_path / "old.json"
    f.write_text(json.dumps({"per_launch_bytes": {"k_render_bwd<false>": 1e9, "k_render_fwd_tile<false>": 1e9},
                             "valu_insts_per_launch": {"k_render_bwd<false>": 1e9}}))
    r = bench.roofline_fields(_args("--traffic", str(f)), PHASES, [6.6e6] * 64, [4.95e6] * 64, 1024, 1024)
    assert r["roofline"]["traffic"] is None and bench.KERNELS["c3"][1] in r["counters_note"]


def test_launcher_command_and_world_check():
    cmd = bench.launch_command(["--gpus", "4", "--steps", "3"], 4)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:]
    assert cmd[-5].endswith("bench.py")
    bench.check_world(2, 2)
    import pytest

    with pytest.raises(SystemExit):
        bench.check_world(8, 1)


def test_launcher_starts_ranks_without_world_size(monkeypatch):
    """`bench.py --gpus 2` without a launcher environment hands over to N ranks before touching the GPU."""
    import subprocess

    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    import pytest

    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and len(calls) == 1 and "--nproc-per-node=2" in calls[0]


def test_counters_of_another_build_are_dropped(tmp_path):
    """counter and pair files record the build id of the library they were captured on
    (profiles/summarize.py, profiles/diag_pairs.py); bench.py drops them when the loaded library's id differs."""
    import json

    a0 = _args()
    t = json.load(open(a0.traffic))
    p = json.load(open(a0.pairs))
    for tag, build in (("same", "b0"), ("other", "b1")):
        tf, pf = tmp_path / f"t_{tag}.json", tmp_path / f"p_{tag}.json"
        tf.write_text(json.dumps(dict(t, build_id=build)))
        pf.write_text(json.dumps(dict(p, build_id=build)))
        r = bench.roofline_fields(_args("--traffic", str(tf), "--pairs", str(pf)), PHASES, [6.6e6] * 64,
                                  [4.95e6] * 64, 1024, 1024, build="b0")
        assert r["library_build"] == "b0"
        if tag == "same":
            assert r["roofline"]["traffic"] is not None and "pairs_per_launch" in r["roofline"]["valu"]
            assert "counters_note" not in r
        else:
            assert r["roofline"]["traffic"] is None and "valu" not in r["roofline"]
            assert "another build" in r["counters_note"] and "b1" in r["counters_note"]


def test_config_names_only_the_collectives_that_run(monkeypatch):
    """at N = 1 the workload names no all-gather / all-reduce and the parallelism says so;
    comm_backend / comm_world_size are what torch.distributed reports (None / 1 without a process group, the
    group's backend and size with one — a world-1 gloo group here, RCCL's 'nccl' on the GPU node)."""
    import torch.distributed as dist

    a = _args()
    c1 = bench.config_fields(a, 1, 64, "none", 6.6e6, 4.95e6, False)
    assert "all-gather" not in c1["workload"] and "all-reduce" not in c1["workload"]
    assert c1["parallelism"] == "1 rank, no collectives"
    assert c1["comm_backend"] is None and c1["comm_world_size"] == 1
    c8 = bench.config_fields(a, 8, 8, "RCCL", 6.6e6, 4.95e6, True)
    assert "all-gather" in c8["workload"] and "RCCL all-gather" in c8["parallelism"]
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(bench._free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        cg = bench.config_fields(a, 1, 64, "gloo", 6.6e6, 4.95e6, False)
        assert cg["comm_backend"] == "gloo" and cg["comm_world_size"] == 1
    finally:
        dist.destroy_process_group()


def test_product_timing_imports_no_test_code():
    """the per-view shading leg runs the product's shading kernels (shading.shade_views), not
    the tests' torch restatement; only the CPU baseline imports the oracle (test infrastructure, as the checker)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "torch_reference" not in src and '"tests"' not in src
    assert src.count("import oracle") == 1


def test_pairs_of_the_diag_build_of_the_same_sources_are_used(tmp_path):
    """the diagnostic library's id is the product's id + "-diag" (csrc/Makefile); its pair counts are
    accepted for the product of the same sources, another build's are not."""
    import json

    a0 = _args()
    t = json.load(open(a0.traffic))
    p = json.load(open(a0.pairs))
    tf, pf = tmp_path / "t.json", tmp_path / "p.json"
    tf.write_text(json.dumps(dict(t, build_id="b0")))
    for pid, ok in (("b0-diag", True), ("b1-diag", False)):
        pf.write_text(json.dumps(dict(p, build_id=pid)))
        r = bench.roofline_fields(_args("--traffic", str(tf), "--pairs", str(pf)), PHASES, [6.6e6] * 64,
                                  [4.95e6] * 64, 1024, 1024, build="b0")
        assert ("pairs_per_launch" in r["roofline"]["valu"]) == ok, pid
