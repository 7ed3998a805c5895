"""Data-parallel view exchange (data_parallel.py, gsplat_amd.h stages 1-2).

The multi-view per-Gaussian backward over V gathered view records must equal
the sum over the V views of the reference-API backward
(_C.rasterize_gaussians_backward, itself pinned to the oracle in
test_gpu_parity.py).  Both sides run the blend backward separately, whose
float atomics add in a run-dependent order, so the bar is the atomic-order
noise (1e-5 relative) far inside the north_star's 1e-4; the densification
statistics must match the per-view densify_stats kernel applied view by view.
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REL = 1e-5


def _views(P, W, H, yaws, seed=0):
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    cam0 = S.make_camera(W, H)
    sc = S.make_scene(P, cam0, seed=seed)
    cams = [S.make_orbit_camera(W, H, y) for y in yaws]
    return sc, cams


def _forward(C, s, t, deg=3):
    e = torch.Tensor([])
    return C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                 s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
                                 t["shs"], deg, s.campos, False, False)


def _full_backward(C, s, t, fwd, dpix, deg=3):
    K, color, radii, geom, binning, img = fwd
    e = torch.Tensor([])
    return C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                          s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], deg,
                                          s.campos, geom, K, binning, img, False)


@pytest.mark.parametrize("yaws,deg", [((0.0,), 3), ((-5.0, 0.0, 5.0), 3), ((-12.0, -3.0, 4.0, 9.0, 15.0), 3),
                                      ((-5.0, 0.0, 5.0), 1)])
def test_multiview_equals_sum_of_view_backwards(yaws, deg):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 20000, 256, 192
    sc, cams = _views(P, W, H, yaws)
    t = G.scene_tensors(sc)
    want = None
    records = []
    stats_ref = [torch.zeros(P, device="cuda") for _ in range(3)]
    for v, cam in enumerate(cams):
        s = G.torch_settings(cam)
        dpix = torch.from_numpy(S.make_cotangent(H, W, 10 + v)).cuda()
        fwd = _forward(C, s, t, deg)
        g = _full_backward(C, s, t, fwd, dpix, deg)
        # (dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations) of this view
        per = [g[3], g[5], g[2], g[6], g[7]]
        want = [x.double().clone() for x in per] if want is None else [a + x.double() for a, x in zip(want, per)]
        C.densify_stats(fwd[2].contiguous(), g[0], stats_ref[0], stats_ref[1], stats_ref[2])
        records.append(DP.view_record(s, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix))
    views = torch.stack(records)
    stats = [torch.zeros(P, device="cuda") for _ in range(3)]
    got = DP.multiview_param_grads(views, t["means3D"], t["shs"], deg, t["scales"], t["rotations"], 1.0,
                                   stats=tuple(stats))
    torch.cuda.synchronize()
    names = ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations")
    for name, a, b in zip(names, got, want):
        assert a.shape == b.shape, name
        assert np.isfinite(a.cpu().numpy()).all(), name
        err = G.rel_err(a.cpu().numpy(), b.cpu().numpy())
        assert err < REL, (name, err)
    # statistics: the same per-view quantities, accumulated view by view
    assert G.rel_err(stats[0].cpu().numpy(), stats_ref[0].cpu().numpy()) < REL
    np.testing.assert_array_equal(stats[1].cpu().numpy(), stats_ref[1].cpu().numpy())
    np.testing.assert_array_equal(stats[2].cpu().numpy(), stats_ref[2].cpu().numpy())


def test_view_record_layout():
    """Word 9 = radius | clamped << 24, zero rows for invisible Gaussians, and
    the 40 camera words closing the record."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 5000, 128, 96
    sc, cams = _views(P, W, H, (7.0,))
    s = G.torch_settings(cams[0])
    t = G.scene_tensors(sc)
    dpix = torch.from_numpy(S.make_cotangent(H, W, 3)).cuda()
    fwd = _forward(C, s, t)
    rec = DP.view_record(s, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix).cpu().numpy()
    rows = rec[:P * 10].reshape(P, 10)
    w9 = rows[:, 9].view(np.uint32)
    radii = fwd[2].cpu().numpy()
    np.testing.assert_array_equal((w9 & 0xFFFFFF).astype(np.int64), np.maximum(radii, 0).astype(np.int64))
    assert (rows[radii <= 0] == 0).all()
    bufs = C.parse_buffers(fwd[3], fwd[4], fwd[5], P, fwd[0], W, H, 16)
    cb = bufs["clamped_bits"].cpu().numpy().astype(np.uint32)
    vis = radii > 0
    np.testing.assert_array_equal(w9[vis] >> 24, cb[vis])
    cam = rec[P * 10:]
    np.testing.assert_array_equal(cam[:16], s.viewmatrix.cpu().numpy().ravel())
    np.testing.assert_array_equal(cam[16:32], s.projmatrix.cpu().numpy().ravel())
    np.testing.assert_array_equal(cam[32:35], s.campos.cpu().numpy())
    assert cam[35] == W and cam[36] == H
    assert cam[37] == np.float32(s.tanfovx) and cam[38] == np.float32(s.tanfovy)


def test_multiview_more_than_64_views():
    """V > 64 views (e.g. 16 ranks x 8 views) through both C
    entries -- the strided record stack and the per-view pointer lists that
    ViewExchange.finish uses.  Beyond 64 the pointers go through a device
    table; the sums are the same: the 70-view result equals the two 35-view
    halves added (atomic-free per-Gaussian sums: only the halves' rounding
    differs), and the two entries agree bit for bit."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 6000, 128, 96
    sc, cams = _views(P, W, H, (-6.0, 0.0, 7.0))
    t = G.scene_tensors(sc)
    base = []
    for v, cam in enumerate(cams):
        s = G.torch_settings(cam)
        dpix = torch.from_numpy(S.make_cotangent(H, W, 30 + v)).cuda()
        fwd = _forward(C, s, t)
        base.append(DP.view_record(s, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix))
    V = 70
    views = torch.stack([base[v % 3] for v in range(V)]).contiguous()
    args = (t["means3D"], t["shs"], 3, t["scales"], t["rotations"], 1.0)
    got = DP.multiview_param_grads(views, *args)
    h1 = DP.multiview_param_grads(views[:35].contiguous(), *args)
    h2 = DP.multiview_param_grads(views[35:].contiguous(), *args)
    torch.cuda.synchronize()
    for a, b1, b2 in zip(got, h1, h2):
        want = (b1.double() + b2.double()).cpu().numpy()
        assert np.isfinite(a.cpu().numpy()).all()
        assert G.rel_err(a.cpu().numpy(), want) < REL
    # the per-view pointer entry (ViewExchange.finish's) over the same 70 views
    e = torch.empty(0, device="cuda")
    M = t["shs"].shape[1]
    outs = (torch.empty((P, 3), device="cuda"), torch.empty((P, M, 3), device="cuda"),
            torch.empty((P, 1), device="cuda"), torch.empty((P, 3), device="cuda"), torch.empty((P, 4), device="cuda"))
    rows = [views[v, :P * DP.VIEW_ROW] for v in range(V)]
    cams_ = [views[v, P * DP.VIEW_ROW:] for v in range(V)]
    C.backward_gaussians_multiview_views(rows, cams_, 0, t["means3D"], t["shs"], 3, t["scales"], t["rotations"], 1.0,
                                         *outs, e, e, e)
    torch.cuda.synchronize()
    for a, b in zip(got, outs):
        assert torch.equal(a.reshape(-1), b.reshape(-1))


@pytest.mark.parametrize("n_streams", [2, 3])
def test_views_on_streams_match_one_stream(n_streams):
    """data_parallel.run_views_on_streams (config 5's step): the views'
    forward + blend backward alternating over HIP streams give the records
    and parameter gradients of the one-stream loop (float-atomic order noise:
    1e-5 relative)."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 30000, 320, 240
    yaws = (-9.0, -3.0, 2.0, 6.0, 11.0)
    sc, cams = _views(P, W, H, yaws)
    t = G.scene_tensors(sc)
    sets = [G.torch_settings(c) for c in cams]
    dpix = [torch.from_numpy(S.make_cotangent(H, W, 50 + v)).cuda() for v in range(len(cams))]

    def step(ns):
        ex = DP.ViewExchange(P, len(cams), "cuda")

        def one(j):
            fwd = _forward(C, sets[j], t)
            ex.add(j, DP.view_record(sets[j], fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix[j]))

        DP.run_views_on_streams(len(cams), one, ns)
        out = ex.finish(sets[0], t["means3D"], t["shs"], t["scales"], t["rotations"])
        return ex.records(), out

    rec1, g1 = step(1)
    rec2, g2 = step(n_streams)
    torch.cuda.synchronize()
    assert G.rel_err(rec2.cpu().numpy(), rec1.cpu().numpy()) < REL
    for a, b in zip(g2, g1):
        assert G.rel_err(a.cpu().numpy(), b.cpu().numpy()) < REL
