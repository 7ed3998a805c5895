"""The C ABI on the GPU without the torch binding (include/gsplat_amd.h,
INTEGRATION.md §2.2): the reference's Rasterizer::forward / ::backward
(base/cr/rasterizer.h:24-84) and the AMR Rasterizer::forward
(amr/cr/rasterizer.h:24-98) replacements driven through ctypes, as a host
without the pybind module would bind them -- torch-allocated device tensors
as plain pointers, gs_buffer resize callbacks that allocate the byte buffers,
and an explicit (non-default) HIP stream.

On config 1's inputs (10k Gaussians, 256 x 256, seed 0) the results equal the
`_C` path's: K, radii, point_list, ranges and the image bit for bit; the AMR
steps' images and render_once bit for bit; the gradients bit for bit except
for the order of the blend backward's float atomics (their last bits are
run-dependent for any two runs, _C against _C included; bounded here at
1e-6 of each tensor's norm).
"""
import ctypes
import os

import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

VP = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
RESIZE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


class GsBuffer(ctypes.Structure):
    _fields_ = [("resize", RESIZE), ("ctx", ctypes.c_void_p)]


def _lib():
    import gaussian_splatting_with_eye_tracking_amd as pkg
    lib = ctypes.CDLL(os.path.join(os.path.dirname(pkg.__file__), "libgsplat_amd.so"))
    fwd = [GsBuffer, GsBuffer, GsBuffer, I, I, I, VP, I, I, VP, VP, VP, VP, VP, F, VP, VP, VP, VP, VP, F, F, I]
    lib.gs_rasterizer_forward.argtypes = fwd + [VP, VP, I, VP]
    lib.gs_rasterizer_backward.argtypes = ([I, I, I, I, VP, I, I, VP, VP, VP, VP, F, VP, VP, VP, VP, VP, F, F, VP,
                                            VP, VP, VP, VP] + [VP] * 9 + [I, VP])
    lib.gs_amr_rasterizer_forward.argtypes = fwd + [I, VP, VP, VP, VP, VP, VP, I, I, VP]
    lib.gs_last_error.restype = ctypes.c_char_p
    for f in (lib.gs_rasterizer_forward, lib.gs_rasterizer_backward, lib.gs_amr_rasterizer_forward):
        f.restype = I
    return lib


class Buffers:
    """Caller-owned byte buffers behind gs_buffer callbacks (the reference's
    resizeFunctional, base/rasterize_points.cu:27-33): each resize allocates a
    torch uint8 device tensor and returns its pointer."""

    def __init__(self, device):
        self.t = {}
        self.cb = {}
        self.device = device

    def buf(self, key):
        def _resize(_ctx, n):
            self.t[key] = torch.empty(max(int(n), 1), dtype=torch.uint8, device=self.device)
            return self.t[key].data_ptr()
        self.cb[key] = RESIZE(_resize)  # (kept alive as long as the buffers)
        return GsBuffer(self.cb[key], None)


def _p(t):
    return VP(t.data_ptr()) if t is not None and t.numel() else VP(0)


def _check(lib, rc, what):
    assert rc >= 0, f"{what}: {lib.gs_last_error().decode()}"
    return rc


def _inputs(P=10_000, W=256, H=256, seed=0):
    sc, cam = G.scene_and_camera(P, W, H, seed)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    return sc, cam, s, t


def test_forward_backward_through_ctypes_match_the_binding():
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    lib = _lib()
    P, W, H = 10_000, 256, 256
    sc, cam, s, t = _inputs(P, W, H)
    e = torch.Tensor([])
    dpix = torch.from_numpy(S.make_cotangent(H, W, 1)).cuda()
    # the binding (torch's current stream)
    K0, col0, rad0, gb0, bb0, ib0 = C.rasterize_gaussians(
        s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e, s.viewmatrix, s.projmatrix,
        s.tanfovx, s.tanfovy, H, W, t["shs"], 3, s.campos, False, False)
    g0 = C.rasterize_gaussians_backward(s.bg, t["means3D"], rad0, e, t["scales"], t["rotations"], 1.0, e,
                                        s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3, s.campos,
                                        gb0, K0, bb0, ib0, False)
    torch.cuda.synchronize()
    # the C ABI through ctypes, on an explicit stream
    stream = torch.cuda.Stream()
    bufs = Buffers(t["means3D"].device)
    with torch.cuda.stream(stream):
        col = torch.empty((3, H, W), device="cuda")
        radii = torch.empty(P, dtype=torch.int32, device="cuda")
        K = _check(lib, lib.gs_rasterizer_forward(
            bufs.buf("geom"), bufs.buf("binning"), bufs.buf("image"), P, 3, 16, _p(s.bg), W, H, _p(t["means3D"]),
            _p(t["shs"]), VP(0), _p(t["opacities"]), _p(t["scales"]), F(1.0), _p(t["rotations"]), VP(0),
            _p(s.viewmatrix), _p(s.projmatrix), _p(s.campos), F(s.tanfovx), F(s.tanfovy), 0, _p(col), _p(radii), 0,
            VP(stream.cuda_stream)), "gs_rasterizer_forward")
        outs = [torch.empty(shape, device="cuda") for shape in ((P, 3), (P, 1), (P, 3), (P, 3), (P, 6), (P, 16, 3),
                                                                (P, 3), (P, 4))]
        m2, op, cl, m3, cv, sh, scl, rot = outs
        _check(lib, lib.gs_rasterizer_backward(
            P, 3, 16, K, _p(s.bg), W, H, _p(t["means3D"]), _p(t["shs"]), VP(0), _p(t["scales"]), F(1.0),
            _p(t["rotations"]), VP(0), _p(s.viewmatrix), _p(s.projmatrix), _p(s.campos), F(s.tanfovx), F(s.tanfovy),
            _p(radii), _p(bufs.t["geom"]), _p(bufs.t["binning"]), _p(bufs.t["image"]), _p(dpix), _p(m2), VP(0),
            _p(op), _p(cl), _p(m3), _p(cv), _p(sh), _p(scl), _p(rot), 0, VP(stream.cuda_stream)),
            "gs_rasterizer_backward")
    stream.synchronize()
    assert K == K0 > 0
    assert torch.equal(radii, rad0)
    assert torch.equal(col, col0)
    d = C.parse_buffers(bufs.t["geom"], bufs.t["binning"], bufs.t["image"], P, K, W, H, 16)
    d0 = C.parse_buffers(gb0, bb0, ib0, P, K0, W, H, 16)
    for k in ("point_list", "ranges", "n_contrib", "accum_alpha"):
        assert torch.equal(d[k], d0[k]), k
    vis = rad0 > 0  # (culled Gaussians' geometry records are never written)
    for k in ("means2D", "conic_opacity", "depths"):
        assert torch.equal(d[k][vis], d0[k][vis]), k
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    mine = dict(zip(names, [m2, cl, op, m3, cv, sh, scl, rot]))
    for n, ref in zip(names, g0):
        assert mine[n].shape == ref.shape, n
        assert G.rel_err(mine[n].cpu().numpy(), ref.cpu().numpy()) < 1e-6, n


def test_amr_forward_through_ctypes_matches_the_binding():
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    lib = _lib()
    P, W, H = 10_000, 256, 256
    sc, cam, s, t = _inputs(P, W, H)
    s = G.torch_settings(cam, amr=True)
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        ref_steps = []
        c, rradii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
        ref_steps.append(c.clone())
        acc = c
        for k in range(1, 5):
            c, _, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, False, s)
            ref_steps.append(c.clone())
            acc = acc + c
        ref_once = _RasterizeGaussians.apply(*args, -2, e, u8, u8, u8, True, s)[0]
    torch.cuda.synchronize()

    def amr_call(bufs, step, pre, out, radii, interp, stream, precomp=None):
        g = bufs.t.get("geom") if step >= 1 else None
        b = bufs.t.get("binning") if step >= 1 else None
        im = bufs.t.get("image") if step >= 1 else None
        return _check(lib, lib.gs_amr_rasterizer_forward(
            bufs.buf("geom") if step < 1 else bufs.buf("unused_g"),
            bufs.buf("binning") if step < 1 else bufs.buf("unused_b"),
            bufs.buf("image") if step < 1 else bufs.buf("unused_i"), P, 3, 16, _p(s.bg), W, H, _p(t["means3D"]),
            _p(t["shs"]), VP(0), _p(t["opacities"]), _p(t["scales"]), F(1.0), _p(t["rotations"]), VP(0),
            _p(s.viewmatrix), _p(s.projmatrix), _p(s.campos), F(s.tanfovx), F(s.tanfovy), 0, step, _p(precomp),
            _p(g), _p(b), _p(im), _p(out), _p(radii), 1 if interp else 0, 0, VP(stream.cuda_stream)),
            f"gs_amr_rasterizer_forward step {step}")

    stream = torch.cuda.Stream()
    bufs = Buffers(t["means3D"].device)
    steps = []
    with torch.cuda.stream(stream):
        radii = torch.empty(P, dtype=torch.int32, device="cuda")
        acc = None
        for k in range(5):
            out = torch.empty((3, H, W), device="cuda")
            rk = torch.empty(P, dtype=torch.int32, device="cuda")
            amr_call(bufs, k, None, out, radii if k == 0 else rk, False, stream, precomp=acc)
            steps.append(out)
            acc = out if acc is None else acc + out
        once = torch.empty((3, H, W), device="cuda")
        once_bufs = Buffers(t["means3D"].device)
        amr_call(once_bufs, -2, None, once, torch.empty(P, dtype=torch.int32, device="cuda"), True, stream)
    stream.synchronize()
    assert torch.equal(radii, rradii)
    for k in range(5):
        assert torch.equal(steps[k], ref_steps[k]), k
    assert torch.equal(once, ref_once)
