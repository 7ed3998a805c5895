"""CPU-side checks of the product path that need no GPU compute:

* the C-ABI library loads and exports every symbol include/gsplat_amd.h
  declares, and its pure-host size/layout helpers are consistent;
* the torch extension loads and exposes the reference's _C surface;
* the drop-in packages expose the reference API with the reference's error
  behaviour, and the product path fails loudly instead of falling back to the
  CPU (there is no CPU path).
"""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "gsplat_amd.h")
LIB = os.path.join(ROOT, "gaussian_splatting_with_eye_tracking_amd", "libgsplat_amd.so")


def _declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(gs_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = _declared_functions()
    for must in ("gs_rasterizer_forward", "gs_rasterizer_backward", "gs_rasterizer_mark_visible",
                 "gs_amr_rasterizer_forward", "gs_simple_knn", "gs_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_carries_the_tree_digest():
    """build.py compiles source_digest() into the library (gs_build_digest);
    check_loaded_digest refuses a library built from other sources."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_b", os.path.join(ROOT, "gaussian_splatting_with_eye_tracking_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    lib = ctypes.CDLL(LIB)
    lib.gs_build_digest.restype = ctypes.c_char_p
    d = lib.gs_build_digest().decode()
    assert re.fullmatch(r"[0-9a-f]{16}", d)
    assert d == b.source_digest() == b.check_loaded_digest()


def test_tuning_keys_round_trip():
    """gs_set_tuning / gs_get_tuning (pure host state): every documented key
    reports its default, a fallback value sticks, a negative value restores
    the default, and an unknown key is refused with a message."""
    lib = ctypes.CDLL(LIB)
    lib.gs_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.gs_get_tuning.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    lib.gs_last_error.restype = ctypes.c_char_p

    def get(k):
        v = ctypes.c_int(-99)
        assert lib.gs_get_tuning(k.encode(), ctypes.byref(v)) == 0, k
        return v.value

    defaults = {k: get(k) for k in ("fwd_variant", "bwd_variant", "amr_variant", "sort_algo", "cull", "hdr_mirror",
                                    "spec_dup", "ritnet_mfma")}
    assert defaults["fwd_variant"] != 0 and defaults["bwd_variant"] != 0 and defaults["amr_variant"] != 0
    assert defaults["cull"] == 1 and defaults["sort_algo"] == 1 and defaults["ritnet_mfma"] == 1
    try:
        for k in ("fwd_variant", "bwd_variant", "amr_variant"):
            assert lib.gs_set_tuning(k.encode(), 0) == 0
            assert get(k) == 0, k
            assert lib.gs_set_tuning(k.encode(), -1) == 0
            assert get(k) == defaults[k], k
    finally:
        for k, v in defaults.items():
            lib.gs_set_tuning(k.encode(), v)
    v = ctypes.c_int(0)
    assert lib.gs_get_tuning(b"no_such_key", ctypes.byref(v)) == -1
    assert b"no_such_key" in lib.gs_last_error()
    assert lib.gs_set_tuning(b"no_such_key", 1) == -1


def test_host_layout_helpers():
    lib = ctypes.CDLL(LIB)
    lib.gs_geom_bytes.restype = ctypes.c_size_t
    lib.gs_image_bytes.restype = ctypes.c_size_t
    lib.gs_binning_bytes.restype = ctypes.c_size_t
    lib.gs_knn_workspace_bytes.restype = ctypes.c_size_t
    # 2: gs_image_view gained the band arrays; 3: gs_geom_view gained drgb;
    # 4: drgb and cov3D moved to an optional tail of the geometry buffer;
    # 5: 48-B grad_accum rows
    assert lib.gs_abi_version() == 7
    g1, g2 = lib.gs_geom_bytes(1000), lib.gs_geom_bytes(2000)
    assert g2 > g1 > 1000 * (4 + 4 + 8 + 16 + 12 + 24 + 1 + 48 + 4 + 48)
    assert lib.gs_image_bytes(1920, 1080, 16) >= 1920 * 1080 * 8 + 120 * 68 * 8
    assert lib.gs_binning_bytes(4096) >= 4096 * 20
    assert lib.gs_knn_workspace_bytes(10000) > 10000 * 16
    # views carve 256-B aligned arrays out of a base pointer (no device access)
    class GeomView(ctypes.Structure):
        _fields_ = [(n, ctypes.c_void_p) for n in ("hdr", "depths", "radii", "means2D", "conic_opacity", "rgb",
                                                   "cov3D", "clamped", "drgb", "tiles_touched", "grad_accum")]
    v = GeomView()
    base = 1 << 20
    assert lib.gs_geom_view_of(ctypes.c_void_p(base), 1000, ctypes.byref(v)) == 0
    ptrs = [getattr(v, f[0]) for f in GeomView._fields_]
    assert ptrs[0] == base and all(p % 256 == 0 for p in ptrs) and len(set(ptrs)) == len(ptrs)
    # the optional tail (drgb, cov3D) follows everything else
    head = [p for f, p in zip(GeomView._fields_, ptrs) if f[0] not in ("drgb", "cov3D")]
    assert head == sorted(head) and v.grad_accum < v.drgb < v.cov3D
    assert v.cov3D + 1000 * 24 - base <= g1


@pytest.mark.parametrize("prefix", ["gs_binning", "gs_amr_binning"])
def test_binning_size_inverse_is_exact(prefix):
    """gs_(amr_)binning_count_of_bytes inverts gs_(amr_)binning_bytes (the AMR
    steps >= 1 recover K from the binning buffer's size instead of a device
    read-back); the AMR layout is larger and keeps the base arrays' offsets."""
    lib = ctypes.CDLL(LIB)
    nbytes = getattr(lib, prefix + "_bytes")
    count = getattr(lib, prefix + "_count_of_bytes")
    nbytes.restype = ctypes.c_size_t
    nbytes.argtypes = [ctypes.c_int]
    count.restype = ctypes.c_int
    count.argtypes = [ctypes.c_size_t]
    lib.gs_binning_bytes.restype = ctypes.c_size_t
    lib.gs_binning_bytes.argtypes = [ctypes.c_int]
    ks = list(range(0, 700)) + [4095, 4096, 4097, 123457, 2205067, 4437743, 22303484]
    prev = -1
    for k in ks:
        b = nbytes(k)
        assert b > prev or k == 0
        assert b >= lib.gs_binning_bytes(k)
        prev = b
        assert count(b) == k, k
    assert count(nbytes(1000) + 1) == -1


def test_torch_extension_surface():
    from gaussian_splatting_with_eye_tracking_amd import _C, native_library_paths
    for n in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible", "amr_rasterize_gaussians",
              "distCUDA2", "parse_buffers", "profile_enable", "profile_read", "set_tuning",
              "set_thread_option"):
        assert hasattr(_C, n), n
    assert _C.abi_version() == 7
    assert all(os.path.exists(p) and p.startswith(ROOT) for p in native_library_paths())


def test_dropin_packages_export_reference_names():
    import diff_gaussian_rasterization as base
    import diff_gaussian_rasterization_amr as amr
    from simple_knn._C import distCUDA2  # noqa: F401
    for m in (base, amr):
        for n in ("GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
                  "_C"):
            assert hasattr(m, n), (m.__name__, n)
    assert base.GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug")
    assert amr.GaussianRasterizationSettings._fields == base.GaussianRasterizationSettings._fields


def _settings():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    e = torch.eye(4)
    return GaussianRasterizationSettings(8, 8, 0.5, 0.5, torch.zeros(3), 1.0, e, e, 3, torch.zeros(3), False, False)


@pytest.mark.parametrize("kw,msg", [
    (dict(), "excatly one of either SHs or precomputed colors"),
    (dict(shs=torch.zeros(1, 16, 3), colors_precomp=torch.zeros(1, 3)), "excatly one"),
    (dict(shs=torch.zeros(1, 16, 3)), "scale/rotation pair or precomputed 3D covariance"),
    (dict(shs=torch.zeros(1, 16, 3), scales=torch.ones(1, 3), rotations=torch.ones(1, 4), cov3D_precomp=torch.ones(1, 6)),
     "exactly one of either scale/rotation"),
])
def test_exactly_one_checks_raise_like_reference(kw, msg):
    """base/.../__init__.py:191-195 raise a bare Exception (before any native call)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    m = torch.zeros(1, 3)
    with pytest.raises(Exception, match=msg):
        GaussianRasterizer(_settings())(means3D=m, means2D=m, opacities=torch.ones(1, 1), **kw)


def test_bad_means3D_shape_raises_runtime_error():
    """rasterize_points.cu:57-59: AT_ERROR -> RuntimeError."""
    from gaussian_splatting_with_eye_tracking_amd import _C
    s = _settings()
    e = torch.Tensor([])
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(s.bg, torch.zeros(4, 2), e, torch.ones(4, 1), e, e, 1.0, e, s.viewmatrix,
                               s.projmatrix, 0.5, 0.5, 8, 8, torch.zeros(4, 16, 3), 3, s.campos, False, False)


def test_no_cpu_fallback():
    """Host tensors are refused loudly: the product path has no CPU route."""
    from diff_gaussian_rasterization import GaussianRasterizer
    m = torch.zeros(5, 3)
    with pytest.raises(RuntimeError, match="HIP device tensor"):
        GaussianRasterizer(_settings())(means3D=m, means2D=m, opacities=torch.ones(5, 1), shs=torch.zeros(5, 16, 3),
                                        scales=torch.ones(5, 3), rotations=torch.ones(5, 4))
    from simple_knn._C import distCUDA2
    with pytest.raises(RuntimeError, match="HIP device tensor"):
        distCUDA2(torch.zeros(5, 3))


def test_amr_wrapper_defaults_match_reference():
    import inspect

    from diff_gaussian_rasterization_amr import GaussianRasterizer
    sig = inspect.signature(GaussianRasterizer.forward)
    assert sig.parameters["foveaStep"].default == 0
    assert sig.parameters["interpolate_image"].default is True
    for n in ("out_color_precomp", "geomBuffer_precomp", "binningBuffer_precomp", "imageBuffer_precomp"):
        assert sig.parameters[n].default is None


def test_new_entry_points_validate_before_any_device_call():
    """Argument errors of the extension entry points come back as negative
    codes with a gs_last_error message, raised on the host before any HIP
    call (so this runs without a GPU)."""
    lib = ctypes.CDLL(LIB)
    lib.gs_last_error.restype = ctypes.c_char_p
    null = ctypes.c_void_p(0)
    # gamma/CLAHE preprocessing: the image must tile into the grid
    rc = lib.gs_eye_preprocess(null, ctypes.c_int(401), ctypes.c_int(640), null, ctypes.c_double(1.5),
                               ctypes.c_int(8), ctypes.c_int(8), null, null, null)
    assert rc < 0 and b"divisible" in lib.gs_last_error()
    # fovea levels: at most 4 discs; the image buffer must hold width x height
    buf = ctypes.create_string_buffer(64)
    c = (ctypes.c_float * 8)()
    r = (ctypes.c_float * 4)(100.0, 50.0, 25.0, 12.0)
    rc = lib.gs_amr_fovea_levels(buf, ctypes.c_size_t(64), ctypes.c_int(256), ctypes.c_int(256), ctypes.c_int(5), c,
                                 r, ctypes.c_int(1), ctypes.c_int(0), null)
    assert rc < 0 and b"0 to 4" in lib.gs_last_error()
    rc = lib.gs_amr_fovea_levels(buf, ctypes.c_size_t(64), ctypes.c_int(256), ctypes.c_int(256), ctypes.c_int(4), c,
                                 r, ctypes.c_int(1), ctypes.c_int(0), null)
    assert rc < 0 and b"too small" in lib.gs_last_error()
    # AMR backward: foveaStep 0 has no image; interpolation only for render_once
    def amr_bwd(step, interp):
        args = [ctypes.c_int(10), ctypes.c_int(3), ctypes.c_int(16), ctypes.c_int(0), null, ctypes.c_int(64),
                ctypes.c_int(64)] + [null] * 4 + [ctypes.c_float(1.0)] + [null] * 5 + [ctypes.c_float(0.5)] * 2 + \
               [null] * 4 + [ctypes.c_int(step), ctypes.c_int(interp)] + [null] * 11 + [ctypes.c_int(0), null]
        return lib.gs_amr_rasterizer_backward(*args)
    assert amr_bwd(0, 0) < 0 and b"renders nothing" in lib.gs_last_error()
    assert amr_bwd(2, 1) < 0 and b"render_once only" in lib.gs_last_error()
    assert amr_bwd(5, 0) < 0 and b"1..4" in lib.gs_last_error()
    # the fused step-and-sum: foveaStep 1..4 only, and the step-0 buffers
    def acc_step(step, geom):
        return lib.gs_amr_accumulate_step(ctypes.c_int(10), null, ctypes.c_int(64), ctypes.c_int(64), null,
                                          ctypes.c_int(step), geom, null, geom, geom, null, ctypes.c_int(0),
                                          ctypes.c_int(-1), null)
    assert acc_step(0, buf) < 0 and b"1..4" in lib.gs_last_error()
    assert acc_step(5, buf) < 0 and b"1..4" in lib.gs_last_error()
    assert acc_step(2, null) < 0 and b"foveaStep 0" in lib.gs_last_error()
    # GSPLAT_AMD_AMR_STEPS_1_TO_4 (steps 1..4 in one launch) passes the step check
    assert acc_step(14, null) < 0 and b"foveaStep 0" in lib.gs_last_error()
    assert acc_step(15, null) < 0 and b"foveaStep 0" in lib.gs_last_error()
    assert lib.gs_set_thread_option(b"amr_step0_unfilled", 0) == 0


def test_extension_entry_points_in_torch_module():
    from gaussian_splatting_with_eye_tracking_amd import _C
    for n in ("amr_rasterize_gaussians_backward", "amr_fovea_levels", "eye_preprocess", "ritnet_conv", "avgpool2",
              "ritnet_head", "label_moments"):
        assert hasattr(_C, n), n
