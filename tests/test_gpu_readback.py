"""GPU: the forward's K read-back modes give identical results.

hdr_mirror 0 copies the header words to pinned host memory behind the tile
scan and waits on an event; 1 lets the scan store them into mapped host memory
(event after the scan); 2 adds a per-call token after a system-scope fence and
the host spins on it (no marker in the stream).  Every mode must produce the
same K, image, radii and binning -- across repeated calls (the token changes
per call, the mirror words are reused), a size change (speculative duplicate
grow / shrink) and the AMR step-0 path (work enqueued between the read's two
halves).
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _forward(sc, cam):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    out = C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], s.scale_modifier,
                                e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
                                t["shs"], s.sh_degree, s.campos, s.prefiltered, s.debug)
    torch.cuda.synchronize()
    K, color, radii = out[0], out[1], out[2]
    return int(K), color.cpu().numpy(), radii.cpu().numpy()


@pytest.mark.parametrize("mode", [2])
def test_readback_modes_match_copy(mode):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    scenes = [G.scene_and_camera(P, W, H, seed) for P, W, H, seed in
              ((10000, 256, 256, 0), (30000, 320, 200, 3), (5000, 256, 256, 1))]
    ref = []
    try:
        C.set_tuning("hdr_mirror", 0)
        for sc, cam in scenes:
            ref.append(_forward(sc, cam))
        C.set_tuning("hdr_mirror", mode)
        for rep in range(3):
            for (sc, cam), (K0, c0, r0) in zip(scenes, ref):
                K, c, r = _forward(sc, cam)
                assert K == K0, (mode, rep, K, K0)
                assert np.array_equal(c, c0), (mode, rep)
                assert np.array_equal(r, r0), (mode, rep)
    finally:
        C.set_tuning("hdr_mirror", 2)


def test_readback_poll_amr_step0():
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    import bench
    W, H, P = 256, 256, 10000
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    dev = torch.device("cuda:0")
    st = bench.raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = bench.device_params(sc, dev, False)
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    a = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)

    def frame():
        with torch.no_grad():
            c_, _r, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
            acc = c_
            for k in range(1, 5):
                c_, _, gb, bb, ib = _RasterizeGaussians.apply(*a, k, acc, gb, bb, ib, False, st)
                acc = acc + c_
        torch.cuda.synchronize()
        return acc.cpu().numpy()

    try:
        C.set_tuning("hdr_mirror", 0)
        ref = frame()
        C.set_tuning("hdr_mirror", 2)
        for _ in range(2):
            assert np.array_equal(frame(), ref)
    finally:
        C.set_tuning("hdr_mirror", 2)
