"""Pin the CPU oracle before trusting it (CPU only).

* against the reference's own Python, via tests/golden/ref_pins.npz (made by
  tools/make_golden.py from /root/reference: utils/sh_utils.py:eval_sh,
  utils/graphics_utils.py:getProjectionMatrix / getWorld2View2 /
  geom_transform_points) -- and directly against /root/reference when it is
  mounted (this container; not the GPU box);
* against its own committed regression vectors G1-G4 (bit-exact);
* against hand-computed known answers of the CUDA-only stages (the
  reference has no tests for those: SURVEY §4).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from gaussian_splatting_with_eye_tracking_amd import synthetic as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = "/root/reference"


def _pins():
    return np.load(os.path.join(GOLD, "ref_pins.npz"))


def _eval_sh_oracle(deg, dirs, sh_c16):
    """oracle SH polynomial; sh_c16 is eval_sh's [N, 3, 16] layout."""
    L = O.lib()
    out = np.zeros((dirs.shape[0], 3), np.float32)
    for i in range(dirs.shape[0]):
        sh = np.ascontiguousarray(sh_c16[i].T)  # -> [16][3]
        d = np.ascontiguousarray(dirs[i])
        o = np.zeros(3, np.float32)
        L.orc_eval_sh(ctypes.c_int(deg), O._p(d), O._p(sh), O._p(o))
        out[i] = o
    return out


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_matches_reference_eval_sh(deg):
    p = _pins()
    got = _eval_sh_oracle(deg, p["sh_dirs"], p["sh_coeffs"])
    ref = p[f"eval_sh_deg{deg}"]
    # same expression order as utils/sh_utils.py:eval_sh in float32: bit-exact
    np.testing.assert_array_equal(got, ref)


def test_projection_matrix_matches_reference():
    p = _pins()
    for prm, ref in zip(p["proj_params"], p["proj"]):
        np.testing.assert_array_equal(S.get_projection_matrix(*prm), ref)


def test_world2view_matches_reference():
    p = _pins()
    for R, t, ref in zip(p["w2v_R"], p["w2v_t"], p["w2v"]):
        np.testing.assert_array_equal(S.get_world2view2(R, t), ref)


def test_means2D_matches_reference_projection():
    """oracle means2D = ndc2Pix(p_proj) with p_proj from geom_transform_points."""
    p = _pins()
    cam = S.make_camera(320, 240)
    np.testing.assert_array_equal(cam.full_proj_transform, p["gtp_full_proj"])
    sc = S.make_scene(1000, cam, seed=3)
    np.testing.assert_array_equal(sc.means3D, p["gtp_points"])
    r = O.preprocess_and_bin(O.settings_from_camera(cam), sc.means3D, sc.opacities, shs=sc.shs, scales=sc.scales,
                             rotations=sc.rotations)
    vis = r.radii > 0
    g = p["gtp_out"].astype(np.float64)
    ref_px = ((g[:, 0] + 1.0) * 320 - 1.0) * 0.5
    ref_py = ((g[:, 1] + 1.0) * 240 - 1.0) * 0.5
    np.testing.assert_allclose(r.means2D[vis, 0], ref_px[vis], atol=2e-3)
    np.testing.assert_allclose(r.means2D[vis, 1], ref_py[vis], atol=2e-3)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted (GPU box)")
def test_pins_regenerate_from_reference():
    """The committed pins are what the reference computes today."""
    import subprocess
    import sys
    import tempfile
    code = (f"import sys; sys.dont_write_bytecode=True; sys.path.insert(0, {REF!r});"
            "import numpy as np, torch; from utils.sh_utils import eval_sh;"
            f"p=np.load({os.path.join(GOLD, 'ref_pins.npz')!r});"
            "r=eval_sh(3, torch.from_numpy(p['sh_coeffs']), torch.from_numpy(p['sh_dirs'])).numpy();"
            "assert np.array_equal(r, p['eval_sh_deg3']); print('ok')")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                         cwd=tempfile.gettempdir())
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr


# ------------------------------------------------------ regression vectors ---
def _regen_inputs(d):
    P, W, H, seed = int(d["P"]), int(d["W"]), int(d["H"]), int(d["seed"])
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=seed)
    dpix = S.make_cotangent(H, W, seed + 1)
    if "shs" in d:
        np.testing.assert_array_equal(sc.shs, d["shs"])
    else:
        assert np.float64(np.asarray(sc.shs, np.float64).sum()) == d["shs_sum"]
        assert np.float64(np.asarray(dpix, np.float64).sum()) == d["dL_dpix_sum"]
    return cam, sc, dpix


@pytest.mark.parametrize("name", ["G1", "G2"])
def test_oracle_regression_base(name):
    d = np.load(os.path.join(GOLD, f"oracle_{name}.npz"))
    cam, sc, dpix = _regen_inputs(d)
    s = O.settings_from_camera(cam, bg=(0.1, 0.2, 0.3))
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    r = O.forward(s, sc.means3D, sc.opacities, **kw)
    assert r.num_rendered == int(d["num_rendered"])
    for k in ("radii", "means2D", "depths", "conic_opacity", "rgb", "tiles_touched", "point_list_keys", "point_list",
              "ranges", "color", "final_T", "n_contrib"):
        np.testing.assert_array_equal(getattr(r, k), d[k], err_msg=k)
    g = O.backward(s, r, sc.means3D, dpix, **kw)
    for k, v in g.items():
        np.testing.assert_array_equal(v, d[k], err_msg=k)


def test_oracle_regression_amr():
    d = np.load(os.path.join(GOLD, "oracle_G3.npz"))
    cam = S.make_camera(256, 256)
    sc = S.make_scene(10000, cam, seed=0)
    s = O.settings_from_camera(cam)
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    acc, radii, st, steps = O.amr_render_foveated(s, kw)
    np.testing.assert_array_equal(st.percentile_values, d["percentile_values"])
    np.testing.assert_array_equal(st.levels, d["levels"])
    np.testing.assert_array_equal(np.stack(steps), d["steps"])
    np.testing.assert_array_equal(acc, d["render"])
    once, _, _ = O.amr_render_once(s, kw)
    np.testing.assert_array_equal(once, d["render_once"])


def test_oracle_regression_knn():
    d = np.load(os.path.join(GOLD, "oracle_G4.npz"))
    dist, morton, idx, boxes = O.knn_intermediates(d["points"])
    np.testing.assert_array_equal(dist, d["dist"])
    np.testing.assert_array_equal(morton, d["morton_sorted"])
    np.testing.assert_array_equal(idx, d["indices_sorted"])
    np.testing.assert_array_equal(boxes, d["boxes"])
