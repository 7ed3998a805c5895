"""PLY scenes on the device: a scene file in the
reference's save_ply layout (scene/gaussian_model.py:177-206) is mapped,
uploaded and activated on the GPU (csrc/train.hip activate_kernel), rendered
through the drop-in rasterizer and checked against the CPU oracle; the flat
training state loaded from it writes the same bytes back.  No reference PLY
fixture exists (the reference ships none); the files are synthetic, written
in the reference's format."""
import numpy as np
import pytest
import torch

import gs_helpers as G

pytestmark = pytest.mark.gpu


def _ply_scene(tmp_path, P=20000, W=320, H=200, seed=3):
    from gaussian_splatting_with_eye_tracking_amd import ply
    sc, cam = G.scene_and_camera(P, W, H, seed)
    path = str(tmp_path / "scene.ply")
    ply.write_ply(path, ply.from_activated(sc.means3D, sc.opacities, sc.scales, sc.rotations, sc.shs))
    return path, cam


def test_device_activation_matches_host(tmp_path):
    from gaussian_splatting_with_eye_tracking_amd import ply
    path, _ = _ply_scene(tmp_path)
    g = ply.read_ply(path)
    d = ply.to_device_inputs(g, "cuda:0")
    h = ply.to_rasterizer_inputs(g)
    for k in ("means3D", "shs"):
        np.testing.assert_array_equal(d[k].cpu().numpy(), h[k].numpy(), err_msg=k)
    for k in ("opacities", "scales", "rotations"):
        np.testing.assert_allclose(d[k].cpu().numpy(), h[k].numpy(), rtol=2e-6, atol=1e-7, err_msg=k)


def test_ply_scene_renders_like_the_oracle(tmp_path):
    import oracle as O
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import ply
    path, cam = _ply_scene(tmp_path)
    g = ply.read_ply(path)
    d = ply.to_device_inputs(g, "cuda:0")
    s = G.torch_settings(cam)
    with torch.no_grad():
        color, radii = GaussianRasterizer(s)(means3D=d["means3D"], means2D=torch.zeros_like(d["means3D"]),
                                             opacities=d["opacities"], shs=d["shs"], scales=d["scales"],
                                             rotations=d["rotations"])
    a = {k: v.cpu().numpy() for k, v in d.items()}  # the device activations, rendered by the oracle
    ref = O.forward(O.settings_from_camera(cam), a["means3D"], a["opacities"], shs=a["shs"], scales=a["scales"],
                    rotations=a["rotations"])
    np.testing.assert_array_equal(radii.cpu().numpy(), ref.radii)
    assert G.image_l1(color.cpu().numpy(), ref.color) < G.IMAGE_L1_TOL


def test_flat_model_round_trips_the_file(tmp_path):
    from gaussian_splatting_with_eye_tracking_amd import ply
    path, _ = _ply_scene(tmp_path, P=5000)
    m = ply.to_flat_model(ply.read_ply(path), spatial_lr_scale=1.0, device="cuda:0")
    assert m.params.is_cuda and m.P == 5000 and m.active_sh_degree == 3
    out = str(tmp_path / "saved.ply")
    ply.write_ply(out, ply.from_flat_model(m))
    assert open(out, "rb").read() == open(path, "rb").read()
