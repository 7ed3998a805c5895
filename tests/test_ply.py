"""Gaussian-scene PLY I/O (gaussian_splatting_with_eye_tracking_amd/ply.py), CPU.

The reference ships no PLY fixture and plyfile is not installed, so the
format is pinned to the reference's writer/reader code
(scene/gaussian_model.py:177-256): property names and order, the channel-major
SH layout, raw (pre-activation) values, and plyfile's header for an all-f4
binary little-endian vertex element.  "Parity unpinned" beyond that spec.
"""
import numpy as np
import pytest
import torch

from gaussian_splatting_with_eye_tracking_amd import ply
from gaussian_splatting_with_eye_tracking_amd import synthetic as S


def _scene(P=257, seed=0):
    cam = S.make_camera(64, 48)
    sc = S.make_scene(P, cam, seed=seed)
    return ply.from_activated(sc.means3D, sc.opacities, sc.scales, sc.rotations, sc.shs), sc


def test_attribute_names_match_reference_order():
    n = ply.attribute_names(3)
    assert len(n) == 62
    assert n[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert n[9] == "f_rest_0" and n[53] == "f_rest_44"
    assert n[54:] == ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]


def test_round_trip_exact_and_header(tmp_path):
    g, _ = _scene()
    p = str(tmp_path / "point_cloud.ply")
    ply.write_ply(p, g)
    raw = open(p, "rb").read()
    head = raw[: raw.index(b"end_header\n") + len(b"end_header\n")].decode()
    assert head.startswith("ply\nformat binary_little_endian 1.0\nelement vertex 257\nproperty float x\n")
    assert len(raw) == len(head) + 257 * 62 * 4
    for mm in (True, False):
        r = ply.read_ply(p, sh_degree=3, mmap=mm)
        for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
            np.testing.assert_array_equal(getattr(r, k), getattr(g, k), err_msg=k)
    assert r.sh_degree == 3


def test_sh_layout_is_channel_major_in_file(tmp_path):
    g, _ = _scene(P=3)
    p = str(tmp_path / "s.ply")
    ply.write_ply(p, g)
    v = np.memmap(p, dtype=np.dtype([(n, "<f4") for n in ply.attribute_names(3)]), mode="r",
                  offset=open(p, "rb").read().index(b"end_header\n") + 11, shape=(3,))
    # f_rest index = channel * 15 + (coefficient - 1)   (features.transpose(1, 2).flatten(1))
    assert v["f_rest_0"][1] == g.features_rest[1, 0, 0]
    assert v["f_rest_15"][1] == g.features_rest[1, 0, 1]
    assert v["f_rest_16"][2] == g.features_rest[2, 1, 1]
    assert v["f_dc_2"][0] == g.features_dc[0, 0, 2]
    assert np.all(v["nx"] == 0)


def test_property_order_extra_props_big_endian_and_ascii(tmp_path):
    g, _ = _scene(P=5)
    names = ply.attribute_names(3)
    cols = dict(zip(names, np.concatenate(
        [g.xyz, np.zeros_like(g.xyz), g.features_dc.transpose(0, 2, 1).reshape(5, -1),
         g.features_rest.transpose(0, 2, 1).reshape(5, -1), g.opacity, g.scaling, g.rotation], axis=1).T))
    order = list(reversed(names)) + ["red"]
    cols["red"] = np.arange(5, dtype=np.float32)
    for fmt, enc in (("binary_big_endian", ">f4"), ("ascii", None)):
        p = str(tmp_path / f"{fmt}.ply")
        with open(p, "wb") as f:
            f.write(f"ply\nformat {fmt} 1.0\ncomment made by test\nelement vertex 5\n".encode())
            f.write("".join(f"property float {n}\n" for n in order).encode() + b"end_header\n")
            if enc:
                arr = np.zeros(5, dtype=[(n, enc) for n in order])
                for n in order:
                    arr[n] = cols[n]
                f.write(arr.tobytes())
            else:
                for i in range(5):
                    f.write((" ".join(repr(float(cols[n][i])) for n in order) + "\n").encode())
        r = ply.read_ply(p, sh_degree=3)
        np.testing.assert_array_equal(r.features_rest, g.features_rest)
        np.testing.assert_array_equal(r.rotation, g.rotation)


def test_sh_degree_mismatch_raises(tmp_path):
    g, _ = _scene(P=4)
    p = str(tmp_path / "s.ply")
    ply.write_ply(p, g)
    with pytest.raises(ValueError):
        ply.read_ply(p, sh_degree=2)


def test_activations_give_the_scene_back(tmp_path):
    g, sc = _scene()
    p = str(tmp_path / "s.ply")
    ply.write_ply(p, g)
    t = ply.to_rasterizer_inputs(ply.read_ply(p))
    np.testing.assert_allclose(t["means3D"].numpy(), sc.means3D)
    np.testing.assert_allclose(t["opacities"].numpy(), sc.opacities, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(t["scales"].numpy(), sc.scales, rtol=1e-5)
    np.testing.assert_allclose(t["rotations"].numpy(), sc.rotations, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(t["shs"].numpy(), sc.shs)
    assert t["shs"].shape == (257, 16, 3) and t["shs"].dtype == torch.float32
