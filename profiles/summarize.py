"""Summarise a rocprofv3 capture (profiles/run_profiles.sh) into committed files:
  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as written by rocprofv3)
  <tag>_pmc.csv            per kernel: dispatches, mean FETCH_SIZE / WRITE_SIZE (KB, raw counter values) and the
                           corrected HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
                           (gfx950: FETCH_SIZE reads 1/2 of a wide coalesced read; MI355X_MICROARCH.md §HBM)
  <tag>_traffic.json       the same per-launch bytes for the blend kernels, read by bench.py for roofline.traffic,
                           and SQ_INSTS_VALU per launch (the VALU roofline), when the valu pass exists
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", f"prof_{tag}")
dst = os.path.dirname(os.path.abspath(__file__))
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))


def agg(path, counter):
    """Mean per launch by kernel, keyed by the kernel name without parameters, 'void ' and 'gsr::'
    (templates keep their arguments: 'k_render_fwd_tile<false>')."""
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].strip()
            if name.startswith("void "):
                name = name[5:]
            d[name].append(float(r["Counter_Value"]))
    return d


f = agg(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
w = agg(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
rows = []
for k in sorted(f, key=lambda k: -sum(f[k]) / len(f[k])):
    fk = sum(f[k]) / len(f[k])
    wk = sum(w.get(k, [0.0])) / max(1, len(w.get(k, [0.0])))
    rows.append((k, len(f[k]), round(fk, 1), round(wk, 1), int((2 * fk + wk) * 1024)))
with open(os.path.join(dst, f"{tag}_pmc.csv"), "w", newline="") as fh:
    wr = csv.writer(fh)
    wr.writerow(["kernel", "dispatches", "FETCH_SIZE_KB", "WRITE_SIZE_KB", "hbm_bytes_per_launch_corrected"])
    wr.writerows(rows)
traffic = {r[0].replace("gsr::", ""): r[4] for r in rows if r[0].startswith("gsr::")}  # ours only
def _build_id():
    """The build id of the library the capture ran (the in-tree product library; bench.py compares it)."""
    import ctypes

    so = os.path.join(os.path.dirname(dst), "threestudio-3dgs_amd", "diff_gaussian_rasterization", "libgsr_hip.so")
    lib = ctypes.CDLL(os.environ.get("GSR_HIP_LIB", so))
    lib.gsr_version.restype = ctypes.c_char_p
    v = lib.gsr_version().decode()
    return v.split(" build ", 1)[1] if " build " in v else "unknown"


summary = {"source": f"profiles/{tag}_pmc.csv", "build_id": _build_id(), "per_launch_bytes": traffic}
vpath = os.path.join(src, "valu", "run_counter_collection.csv")
if os.path.exists(vpath):
    v = agg(vpath, "SQ_INSTS_VALU")
    wv = agg(vpath, "SQ_WAVES")
    summary["valu_insts_per_launch"] = {k.replace("gsr::", ""): round(sum(x) / len(x)) for k, x in v.items()
                                        if k.startswith("gsr::")}
    summary["waves_per_launch"] = {k.replace("gsr::", ""): round(sum(x) / len(x)) for k, x in wv.items()
                                   if k.startswith("gsr::")}
    with open(os.path.join(dst, f"{tag}_valu.csv"), "w", newline="") as fh:
        wr = csv.writer(fh)
        wr.writerow(["kernel", "dispatches", "SQ_INSTS_VALU_per_launch", "SQ_WAVES_per_launch"])
        for k in sorted(v, key=lambda k: -sum(v[k]) / len(v[k])):
            wr.writerow([k, len(v[k]), round(sum(v[k]) / len(v[k])), round(sum(wv.get(k, [0])) / max(1, len(wv.get(k, [0]))))])
json.dump(summary, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
print("\n".join(f"{r[0]:40s} {r[4] / 1e6:10.1f} MB/launch" for r in rows[:12]))
