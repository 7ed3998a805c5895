"""Gaussian-scene PLY I/O.

The reference stores a trained scene with plyfile (scene/gaussian_model.py:
177-256): one binary little-endian `vertex` element of float32 properties in
the order of construct_list_of_attributes (:177-189)

    x y z nx ny nz f_dc_0..2 f_rest_0..(3*(D+1)^2-4) opacity scale_0..2 rot_0..3

holding the *raw* parameters: SH with the file's channel-major layout
(features.transpose(1, 2).flatten(), :195-196), logit opacity, log scales and
unnormalised quaternions.  plyfile is not available here, so this module
parses the PLY header itself and maps the payload with a numpy structured
dtype (no per-vertex Python work; np.memmap for large scenes); it accepts any
property order and extra properties, like the reference's name-based lookup
(:222-245).

`to_rasterizer_inputs` applies the activations the reference's model
getters apply before rasterizing (scene/gaussian_model.py:93-113,
gaussian_renderer/__init__.py:57-78): exp(scale), sigmoid(opacity),
normalize(rotation), SH as [P, (D+1)^2, 3].
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
    "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


@dataclass
class GaussianPly:
    """Raw (pre-activation) parameters, the reference's nn.Parameters."""
    xyz: np.ndarray            # [P, 3]
    features_dc: np.ndarray    # [P, 1, 3]
    features_rest: np.ndarray  # [P, (D+1)^2 - 1, 3]
    opacity: np.ndarray        # [P, 1]  logit
    scaling: np.ndarray        # [P, 3]  log
    rotation: np.ndarray       # [P, 4]  unnormalised (w, x, y, z)

    @property
    def P(self) -> int:
        return self.xyz.shape[0]

    @property
    def sh_degree(self) -> int:
        return int(round(np.sqrt(self.features_rest.shape[1] + 1))) - 1


def attribute_names(sh_degree: int) -> list[str]:
    """scene/gaussian_model.py:177-189."""
    n_rest = 3 * (sh_degree + 1) ** 2 - 3
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)] +
            [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"] + [f"scale_{i}" for i in range(3)] +
            [f"rot_{i}" for i in range(4)])


def _read_header(f):
    line = f.readline()
    if line.strip() != b"ply":
        raise ValueError("not a PLY file")
    fmt = None
    elements = []  # (name, count, [(prop, dtype)])
    while True:
        line = f.readline()
        if not line:
            raise ValueError("truncated PLY header")
        tok = line.decode("ascii").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            if tok[1] == "list":
                raise ValueError("list properties are not supported in Gaussian scenes")
            elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
        elif tok[0] == "end_header":
            return fmt, elements, f.tell()


def read_ply(path: str, sh_degree: int | None = None, mmap: bool = True) -> GaussianPly:
    """scene/gaussian_model.py:213-256 (load_ply), raw parameters as float32."""
    with open(path, "rb") as f:
        fmt, elements, offset = _read_header(f)
    if fmt not in ("binary_little_endian", "binary_big_endian", "ascii"):
        raise ValueError(f"unsupported PLY format {fmt}")
    if not elements or elements[0][0] != "vertex":
        raise ValueError("first PLY element must be 'vertex'")
    _, count, props = elements[0]
    endian = ">" if fmt == "binary_big_endian" else "<"
    dtype = np.dtype([(n, endian + t) for n, t in props])
    if fmt == "ascii":
        with open(path, "rb") as f:
            f.seek(offset)
            flat = np.loadtxt(f, max_rows=count, ndmin=2)
        v = np.zeros(count, dtype=dtype)
        for i, (n, _) in enumerate(props):
            v[n] = flat[:, i]
    elif mmap:
        v = np.memmap(path, dtype=dtype, mode="r", offset=offset, shape=(count,))
    else:
        with open(path, "rb") as f:
            f.seek(offset)
            v = np.fromfile(f, dtype=dtype, count=count)
    names = set(v.dtype.names)

    def col(n):
        return np.asarray(v[n], dtype=np.float32)

    def sorted_prefix(prefix):
        ks = [n for n in v.dtype.names if n.startswith(prefix)]
        return sorted(ks, key=lambda x: int(x.split("_")[-1]))

    xyz = np.stack([col("x"), col("y"), col("z")], axis=1)
    opacity = col("opacity")[:, None]
    dc = np.stack([col(f"f_dc_{i}") for i in range(3)], axis=1)  # [P, 3] channels
    rest_names = sorted_prefix("f_rest_")
    n_coef = (len(rest_names) + 3) // 3
    if sh_degree is not None and len(rest_names) != 3 * (sh_degree + 1) ** 2 - 3:
        raise ValueError(f"{len(rest_names)} f_rest properties do not match SH degree {sh_degree}")  # :232
    rest = (np.stack([col(n) for n in rest_names], axis=1) if rest_names else np.zeros((count, 0), np.float32))
    rest = rest.reshape(count, 3, n_coef - 1).transpose(0, 2, 1)  # (P, F, coeffs) -> [P, coeffs, 3]
    scales = np.stack([col(n) for n in sorted_prefix("scale_")], axis=1)
    rots = np.stack([col(n) for n in sorted_prefix("rot")], axis=1)
    if "x" not in names or scales.shape[1] != 3 or rots.shape[1] != 4:
        raise ValueError("missing Gaussian properties")
    return GaussianPly(xyz=np.ascontiguousarray(xyz), features_dc=np.ascontiguousarray(dc[:, None, :]),
                       features_rest=np.ascontiguousarray(rest), opacity=np.ascontiguousarray(opacity),
                       scaling=np.ascontiguousarray(scales), rotation=np.ascontiguousarray(rots))


def write_ply(path: str, g: GaussianPly) -> None:
    """scene/gaussian_model.py:191-206 (save_ply): binary little endian, the
    header plyfile writes for an all-'f4' vertex element, normals zero."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    P = g.P
    names = attribute_names(g.sh_degree)
    f_dc = g.features_dc.transpose(0, 2, 1).reshape(P, -1)      # transpose(1, 2).flatten(1)
    f_rest = g.features_rest.transpose(0, 2, 1).reshape(P, -1)
    cols = np.concatenate([g.xyz, np.zeros_like(g.xyz), f_dc, f_rest, g.opacity, g.scaling, g.rotation],
                          axis=1).astype("<f4")
    assert cols.shape[1] == len(names)
    header = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % P
    header += "".join(f"property float {n}\n" for n in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(np.ascontiguousarray(cols).tobytes())


def to_rasterizer_inputs(g: GaussianPly, device=None):
    """Activated tensors for GaussianRasterizer.forward (float32):
    means3D, opacities = sigmoid, scales = exp, rotations = normalize
    (scene/gaussian_model.py:93-113), shs = cat(dc, rest) [P, (D+1)^2, 3]."""
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    xyz, op, sc, rot = t(g.xyz), t(g.opacity), t(g.scaling), t(g.rotation)
    shs = torch.cat([t(g.features_dc), t(g.features_rest)], dim=1)
    out = dict(means3D=xyz, opacities=torch.sigmoid(op), scales=torch.exp(sc),
               rotations=torch.nn.functional.normalize(rot), shs=shs)
    if device is not None:
        out = {k: v.to(device, non_blocking=True) for k, v in out.items()}
    return out


def to_device_inputs(g: GaussianPly, device):
    """The device path of `to_rasterizer_inputs`: the raw groups are uploaded
    once (one host -> device copy each; the payload is memory-mapped) and
    activated on the GPU by the HIP activation kernel of the training step
    (csrc/train.hip activate_kernel: exp / sigmoid / normalize / SH concat in
    one launch) -- the rasterizer inputs never exist on the host."""
    import torch
    from . import _C
    dev = torch.device(device)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    dc, rest, op, sc, rot = up(g.features_dc), up(g.features_rest), up(g.opacity), up(g.scaling), up(g.rotation)
    P, M = g.P, 1 + g.features_rest.shape[1]
    out = dict(means3D=up(g.xyz), opacities=torch.empty((P, 1), device=dev),
               scales=torch.empty((P, 3), device=dev), rotations=torch.empty((P, 4), device=dev),
               shs=torch.empty((P, M, 3), device=dev))
    _C.activate(dc, rest, op, sc, rot, out["shs"], out["opacities"], out["scales"], out["rotations"])
    return out


def to_flat_model(g: GaussianPly, spatial_lr_scale: float, device, opt=None):
    """load_ply (scene/gaussian_model.py:208-256) into the flat HBM training
    state (training.FlatGaussianModel): the raw groups, uploaded as stored."""
    import torch
    from .training import FlatGaussianModel
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    raw = {"xyz": up(g.xyz), "f_dc": up(g.features_dc), "f_rest": up(g.features_rest), "opacity": up(g.opacity),
           "scaling": up(g.scaling), "rotation": up(g.rotation)}
    m = FlatGaussianModel(raw, g.sh_degree, spatial_lr_scale, opt=opt, device=device)
    m.active_sh_degree = g.sh_degree  # load_ply (:255)
    return m


def from_flat_model(model) -> GaussianPly:
    """save_ply's inputs (scene/gaussian_model.py:191-206) from the flat device
    buffer: one device -> host copy of all parameter segments."""
    from .training import GROUPS, group_row_shape
    host = model.params.detach().cpu().numpy()
    v, lo = {}, 0
    for g, end in zip(GROUPS, model.seg_end):
        v[g] = host[lo:end].reshape((model.P,) + group_row_shape(g, model.max_sh_degree))
        lo = end
    return GaussianPly(xyz=v["xyz"], features_dc=v["f_dc"], features_rest=v["f_rest"], opacity=v["opacity"],
                       scaling=v["scaling"], rotation=v["rotation"])


def from_activated(means3D, opacities, scales, rotations, shs) -> GaussianPly:
    """Inverse activations (logit, log) -- for writing synthetic scenes."""
    op = np.clip(np.asarray(opacities, np.float64), 1e-7, 1 - 1e-7)
    shs = np.asarray(shs, np.float32)
    return GaussianPly(xyz=np.asarray(means3D, np.float32), features_dc=shs[:, :1, :].copy(),
                       features_rest=shs[:, 1:, :].copy(), opacity=np.log(op / (1 - op)).astype(np.float32),
                       scaling=np.log(np.asarray(scales, np.float64)).astype(np.float32),
                       rotation=np.asarray(rotations, np.float32))
