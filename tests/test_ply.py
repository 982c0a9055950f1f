"""Gaussian-scene PLY I/O (threestudio-3dgs_amd/gaussian_ply.py) against the reference's file layout
(geometry/gaussian_io.py:36-172, written by plyfile — absent here; the layout is restated from the
reference's attribute list and plyfile's binary header format)."""
import os

import numpy as np
import pytest

import gaussian_ply as gp


def _raw(P, D, seed=0):
    rng = np.random.default_rng(seed)
    K = (D + 1) ** 2
    return dict(xyz=rng.normal(size=(P, 3)).astype(np.float32),
                features_dc=rng.normal(size=(P, 1, 3)).astype(np.float32),
                features_rest=rng.normal(size=(P, K - 1, 3)).astype(np.float32),
                opacity=rng.normal(size=(P, 1)).astype(np.float32),
                scaling=rng.normal(size=(P, 3)).astype(np.float32) - 4,
                rotation=rng.normal(size=(P, 4)).astype(np.float32))


def test_attribute_list_matches_reference_layout():
    names = gp.attribute_names(3, 45)
    assert names[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert names[9] == "f_rest_0" and names[53] == "f_rest_44" and len(names) == 62
    assert names[-8:] == ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]


@pytest.mark.parametrize("D", [0, 1, 3])
def test_round_trip_and_byte_layout(tmp_path, D):
    raw = _raw(257, D, seed=D)
    path = os.path.join(tmp_path, "scene.ply")
    gp.save_ply(path, raw["xyz"], raw["features_dc"], raw["features_rest"], raw["opacity"], raw["scaling"],
                raw["rotation"])
    blob = open(path, "rb").read()
    head, body = blob.split(b"end_header\n", 1)
    lines = head.decode().splitlines()
    assert lines[:3] == ["ply", "format binary_little_endian 1.0", "element vertex 257"]
    nprop = 6 + 3 + 3 * ((D + 1) ** 2 - 1) + 1 + 3 + 4
    assert len(lines) == 3 + nprop and all(line.startswith("property float ") for line in lines[3:])
    assert len(body) == 257 * nprop * 4
    rec = np.frombuffer(body, "<f4").reshape(257, nprop)
    # channel-major SH flattening: f_rest index = channel * (K - 1) + coefficient (gaussian_io.py:61-68)
    K1 = (D + 1) ** 2 - 1
    if K1:
        np.testing.assert_array_equal(rec[:, 9 + 1 * K1 + 0], raw["features_rest"][:, 0, 1])
    np.testing.assert_array_equal(rec[:, 3:6], 0)
    back = gp.load_ply(path, D)
    for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
        np.testing.assert_array_equal(back[k], raw[k], err_msg=k)
    assert back["active_sh_degree"] == D


def test_ascii_big_endian_and_shuffled_properties(tmp_path):
    raw = _raw(5, 1, seed=3)
    names = gp.attribute_names(3, 9)
    P = 5
    f_dc = raw["features_dc"].transpose(0, 2, 1).reshape(P, -1)
    f_rest = raw["features_rest"].transpose(0, 2, 1).reshape(P, -1)
    table = np.concatenate([raw["xyz"], np.zeros((P, 3), np.float32), f_dc, f_rest, raw["opacity"], raw["scaling"],
                            raw["rotation"]], 1)
    perm = np.random.default_rng(0).permutation(len(names))
    for fmt in ("ascii", "binary_big_endian"):
        path = os.path.join(tmp_path, f"{fmt}.ply")
        head = ["ply", f"format {fmt} 1.0", "comment made by a test", f"element vertex {P}"]
        head += [f"property {'double' if i % 2 else 'float'} {names[i]}" for i in perm] + ["end_header"]
        with open(path, "wb") as f:
            f.write(("\n".join(head) + "\n").encode())
            if fmt == "ascii":
                for r in table[:, perm]:
                    f.write((" ".join(repr(float(x)) for x in r) + "\n").encode())
            else:
                dt = np.dtype([(names[i], ">f8" if i % 2 else ">f4") for i in perm])
                rec = np.zeros(P, dt)
                for i in perm:
                    rec[names[i]] = table[:, i]
                f.write(rec.tobytes())
        back = gp.load_ply(path, 1)
        for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
            np.testing.assert_array_equal(back[k], raw[k], err_msg=f"{fmt} {k}")


def test_sh_degree_mismatch_raises(tmp_path):
    raw = _raw(4, 1)
    path = os.path.join(tmp_path, "d1.ply")
    gp.save_ply(path, raw["xyz"], raw["features_dc"], raw["features_rest"], raw["opacity"], raw["scaling"],
                raw["rotation"])
    with pytest.raises(AssertionError):
        gp.load_ply(path, 3)


def test_rasterizer_inputs_activations():
    raw = _raw(50, 3)
    raw["features_dc"][0, 0, 0] = 5.0
    raw["active_sh_degree"] = 3
    x = gp.rasterizer_inputs(raw)
    np.testing.assert_allclose(np.linalg.norm(x["rotations"], axis=1), 1, rtol=1e-6)
    np.testing.assert_allclose(x["scales"], np.exp(raw["scaling"]), rtol=1e-6)
    assert x["shs"].shape == (50, 16, 3) and x["shs"][0, 0, 0] == 2.0  # color_clip
    assert ((x["opacities"] > 0) & (x["opacities"] < 1)).all()


@pytest.mark.gpu
def test_rendering_a_loaded_scene_equals_the_direct_scene(tmp_path):
    """A scene written and read back renders the same image (SH-3 path, the reason PLY I/O matters)."""
    import gsr_synthetic as gs
    from gsr_testutil import gpu_render, make_camera

    scene = gs.make_scene(3000, sh_degree=3, seed=11)
    raw = dict(xyz=scene["means3D"], features_dc=scene["shs"][:, :1], features_rest=scene["shs"][:, 1:],
               opacity=np.log(scene["opacities"] / (1 - scene["opacities"])), scaling=np.log(scene["scales"]),
               rotation=scene["rotations"])
    path = os.path.join(tmp_path, "s.ply")
    gp.save_ply(path, **raw)
    x = gp.rasterizer_inputs(gp.load_ply(path, 3), color_clip=1e9)
    loaded = dict(scene)
    loaded.update({k: x[k] for k in ("means3D", "scales", "rotations", "opacities", "shs")})
    cam = make_camera(128, 96)
    bg = np.ones(3, np.float32)
    a = gpu_render(scene, cam, bg)
    b = gpu_render(loaded, cam, bg)
    # exp(log(s)) and sigmoid(logit(o)) round-trip to within an ulp: the images agree to the parity bar
    np.testing.assert_allclose(a["color"], b["color"], atol=1e-5)
    np.testing.assert_allclose(a["alpha"], b["alpha"], atol=1e-5)
