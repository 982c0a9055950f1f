"""Gaussian-scene PLY I/O with the reference's attribute layout, without `plyfile`.

The reference saves / loads 3DGS scenes through `plyfile` (geometry/gaussian_io.py:36-172,
`GaussianIO.construct_list_of_attributes` / `save_ply` / `load_ply`); `plyfile` is not installed here, so
this module reads and writes the same files directly with numpy:

    one element ``vertex`` with float32 properties, in this order
        x y z nx ny nz f_dc_0..f_dc_{3-1} f_rest_0..f_rest_{3 (D+1)^2 - 3 - 1} opacity scale_0..2 rot_0..3
    f_dc / f_rest flattened channel-major: features (P, K, 3) -> transpose(1, 2) -> (P, 3 K)
    (gaussian_io.py:52-84); normals written as zeros.

Writing produces ``format binary_little_endian 1.0`` (plyfile's default, as ``PlyData([el]).write``);
reading accepts binary little/big endian and ASCII, any property order, and float / double / int
property types.  Loading returns the *raw* (pre-activation) parameters like ``load_ply`` stores them
(gaussian_io.py:86-172; ``active_sh_degree = max_sh_degree``, :172) — the only path that yields an SH-3
scene — and ``rasterizer_inputs`` applies the geometry getters' activations (exp scale, normalised
quaternion, sigmoid opacity, concatenated SH; geometry/gaussian_base.py:371-411) so a loaded scene can be
fed to ``GaussianRasterizer`` / ``rasterize_views``.
"""
from __future__ import annotations

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
    "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def attribute_names(n_dc: int = 3, n_rest: int = 45) -> list[str]:
    """`construct_list_of_attributes` (geometry/gaussian_io.py:37-49) for n_dc = 3 DC and n_rest
    rest coefficients (3 ((D+1)^2 - 1))."""
    names = ["x", "y", "z", "nx", "ny", "nz"]
    names += [f"f_dc_{i}" for i in range(n_dc)]
    names += [f"f_rest_{i}" for i in range(n_rest)]
    names += ["opacity"] + [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]
    return names


def save_ply(path: str, xyz, features_dc, features_rest, opacity, scaling, rotation) -> None:
    """`GaussianIO.save_ply` (geometry/gaussian_io.py:51-84): raw parameters xyz (P, 3),
    features_dc (P, 1, 3), features_rest (P, K-1, 3), opacity (P, 1), scaling (P, 3), rotation (P, 4);
    numpy arrays or tensors."""
    def arr(x):
        if hasattr(x, "detach"):
            x = x.detach().cpu().numpy()
        return np.asarray(x, dtype=np.float32)

    xyz = arr(xyz)
    P = xyz.shape[0]
    f_dc = arr(features_dc).reshape(P, -1, 3).transpose(0, 2, 1).reshape(P, -1)
    f_rest = arr(features_rest).reshape(P, -1, 3).transpose(0, 2, 1).reshape(P, -1)
    cols = [xyz, np.zeros_like(xyz), f_dc, f_rest, arr(opacity).reshape(P, 1), arr(scaling).reshape(P, 3),
            arr(rotation).reshape(P, 4)]
    data = np.ascontiguousarray(np.concatenate(cols, axis=1), dtype="<f4")
    names = attribute_names(f_dc.shape[1], f_rest.shape[1])
    assert data.shape[1] == len(names)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {P}"]
    header += [f"property float {n}" for n in names] + ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(data.tobytes())


def _read_header(f):
    if f.readline().strip() != b"ply":
        raise ValueError("not a PLY file")
    fmt, elements = None, []
    while True:
        line = f.readline()
        if not line:
            raise ValueError("PLY header without end_header")
        tok = line.decode("ascii", errors="replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append({"name": tok[1], "count": int(tok[2]), "props": []})
        elif tok[0] == "property":
            if tok[1] == "list":
                raise ValueError("list properties are not supported (Gaussian scenes have none)")
            elements[-1]["props"].append((tok[2], _PLY_TYPES[tok[1]]))
        elif tok[0] == "end_header":
            break
    return fmt, elements


def read_vertices(path: str) -> dict[str, np.ndarray]:
    """Every property of the first element (``plydata.elements[0]``) as a 1-D array."""
    with open(path, "rb") as f:
        fmt, elements = _read_header(f)
        el = elements[0]
        if fmt == "ascii":
            rows = [f.readline().split() for _ in range(el["count"])]
            table = np.array(rows, dtype=np.float64).reshape(el["count"], len(el["props"]))
            return {n: table[:, i].astype(t) for i, (n, t) in enumerate(el["props"])}
        order = "<" if fmt == "binary_little_endian" else ">"
        if fmt not in ("binary_little_endian", "binary_big_endian"):
            raise ValueError(f"unknown PLY format {fmt}")
        dt = np.dtype([(n, order + t) for n, t in el["props"]])
        rec = np.frombuffer(f.read(dt.itemsize * el["count"]), dtype=dt, count=el["count"])
        return {n: rec[n].astype(rec[n].dtype.newbyteorder("=")) for n, _ in el["props"]}


def load_ply(path: str, max_sh_degree: int) -> dict:
    """`GaussianIO.load_ply` (geometry/gaussian_io.py:86-172) without the nn.Parameter / device moves:
    raw xyz (P, 3), features_dc (P, 1, 3), features_rest (P, (D+1)^2 - 1, 3), opacity (P, 1),
    scaling (P, S), rotation (P, R) float32, and active_sh_degree = max_sh_degree."""
    v = read_vertices(path)
    xyz = np.stack([v["x"], v["y"], v["z"]], axis=1).astype(np.float32)
    P = xyz.shape[0]
    opacities = np.asarray(v["opacity"], np.float32)[:, None]
    features_dc = np.zeros((P, 3, 1), np.float32)
    for c in range(3):
        features_dc[:, c, 0] = v[f"f_dc_{c}"]

    def by_index(prefix):
        names = sorted((n for n in v if n.startswith(prefix)), key=lambda x: int(x.split("_")[-1]))
        return np.stack([v[n] for n in names], axis=1).astype(np.float32) if names else np.zeros((P, 0), np.float32)

    if max_sh_degree > 0:
        extra = by_index("f_rest_")
        if extra.shape[1] != 3 * (max_sh_degree + 1) ** 2 - 3:
            raise AssertionError(f"expected {3 * (max_sh_degree + 1) ** 2 - 3} f_rest properties, found "
                                 f"{extra.shape[1]}")
        features_rest = extra.reshape(P, 3, (max_sh_degree + 1) ** 2 - 1).transpose(0, 2, 1)
    else:
        features_rest = features_dc[:, :, 1:].transpose(0, 2, 1)
    return {
        "xyz": xyz,
        "features_dc": np.ascontiguousarray(features_dc.transpose(0, 2, 1)),
        "features_rest": np.ascontiguousarray(features_rest),
        "opacity": opacities,
        "scaling": by_index("scale_"),
        "rotation": by_index("rot"),
        "active_sh_degree": max_sh_degree,
    }


def rasterizer_inputs(raw: dict, color_clip: float = 2.0) -> dict:
    """The geometry getters' activations (geometry/gaussian_base.py:371-411): means3D = xyz,
    scales = exp(scaling), rotations = rotation / |rotation|, opacities = sigmoid(opacity),
    shs = cat(clip(features_dc, -color_clip, color_clip), features_rest) (color_clip default 2.0, :216)
    — float32 numpy, ready for the rasterizer."""
    rot = raw["rotation"].astype(np.float64)
    rot = rot / np.maximum(np.linalg.norm(rot, axis=1, keepdims=True), 1e-12)
    return {
        "means3D": raw["xyz"].astype(np.float32),
        "scales": np.exp(raw["scaling"].astype(np.float64)).astype(np.float32),
        "rotations": rot.astype(np.float32),
        "opacities": (1.0 / (1.0 + np.exp(-raw["opacity"].astype(np.float64)))).astype(np.float32),
        "shs": np.ascontiguousarray(np.concatenate([np.clip(raw["features_dc"], -color_clip, color_clip),
                                                    raw["features_rest"]], axis=1),
                                    dtype=np.float32),
        "sh_degree": int(raw["active_sh_degree"]),
    }
