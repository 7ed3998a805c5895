"""In-tree build of the native pieces (no JIT cache, no pip install).

* ``libgsplat_amd.so``  -- every HIP kernel + the C ABI (include/gsplat_amd.h),
  compiled with ``hipcc --offload-arch=gfx950``.  No torch dependency.
* ``_C.<abi>.so``       -- the PyTorch binding (csrc/torch_ext.cpp), a thin
  C++ layer that mirrors the reference's ``rasterize_points.cu`` on top of
  the C ABI (tensors -> raw pointers, resize callbacks, current HIP stream).

Both land next to this file so they travel with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
ROOT = os.path.dirname(PKG)
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libgsplat_amd.so")
HIP_SOURCES = ["preprocess.hip", "binning.hip", "render.hip", "backward.hip", "multiview.hip", "amr.hip", "knn.hip",
               "loss.hip", "train.hip", "ritnet.hip", "eye_preprocess.hip", "gs_api.cpp"]
ARCH = os.environ.get("GSAMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off is part of the parity contract (see gs_device.cuh).
# -fno-slp-vectorize: the SLP pass packs independent f32 ops into v_pk_* and then
# needs v_mov pairs to form the operand registers; in the blend loops that cost
# more than it saved (render_bwd 0.90 -> 0.68 ms at config 2).
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", "-munsafe-fp-atomics",
             "-fno-slp-vectorize",
             "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}"]
# Per-source flags after HIP_FLAGS: the backward passes' gradients are held
# to a tolerance (1e-4; tests/test_gpu_multiview.py 1e-5 against the per-view
# sum), so they compile with reciprocal math (and the multi-view kernel with
# FMA contraction too: 30 % fewer VALU instructions per view);
# everything on the keys / images keeps the exact contract above.
SOURCE_FLAGS = {"multiview.hip": ["-ffp-contract=fast", "-freciprocal-math", "-fapprox-func"],
                "backward.hip": ["-freciprocal-math", "-fapprox-func"]}
if os.environ.get("GSAMD_EXACT_BWD"):  # diagnostic builds: the backward passes under the exact contract too
    SOURCE_FLAGS = {}
# extra flags for code-generation experiments (e.g. GSAMD_EXTRA_HIPFLAGS=-fno-slp-vectorize)
HIP_FLAGS += shlex.split(os.environ.get("GSAMD_EXTRA_HIPFLAGS", ""))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(shlex.quote(c) for c in cmd)}\n"
                           f"{r.stdout}\n{r.stderr}")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".cuh"))]
    return hs + [os.path.join(INCLUDE, "gsplat_amd.h")]


DIGEST_STAMP = os.path.join(BUILD, "digest.txt")


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def _object_digest(src: str, digest: str) -> str:
    """What one object is built from: its source, every header, the flags
    (and, for gs_api.cpp, the library digest it embeds)."""
    import hashlib
    h = hashlib.sha256()
    for f in [os.path.join(CSRC, src)] + sorted(_headers()):
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + fh.read())
    h.update(" ".join(f for f in HIP_FLAGS + SOURCE_FLAGS.get(src, []) if not f.startswith("-I")).encode())
    if src == "gs_api.cpp":
        h.update(digest.encode())
    return h.hexdigest()[:16]


def build_hip_lib(jobs: int = 8, verbose: bool = False) -> str:
    """Compile every HIP source and link libgsplat_amd.so.  Rebuild rule:
    content digests, not file times -- each object is rebuilt when the digest
    of its source + headers + flags differs from the stamp written next to it
    (_build/<src>.o.digest), and gs_api.cpp compiles the library digest
    (source_digest) in as gs_build_digest() (-DGSAMD_DIGEST), so a loaded
    library reports exactly the sources it was built from
    (check_loaded_digest)."""
    os.makedirs(BUILD, exist_ok=True)
    digest = source_digest()
    objs = []
    todo = []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src + ".o")
        objs.append(o)
        od = _object_digest(src, digest)
        if not os.path.exists(o) or _read(o + ".digest") != od:
            extra = [f"-DGSAMD_DIGEST=\"{digest}\""] if src == "gs_api.cpp" else []
            todo.append((o, od, [HIPCC] + HIP_FLAGS + SOURCE_FLAGS.get(src, []) + extra + ["-x", "hip", "-c", s, "-o", o]))
    if todo:
        def one(t):
            o, od, cmd = t
            _run(cmd)
            with open(o + ".digest", "w") as f:
                f.write(od + "\n")
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for f in [ex.submit(one, t) for t in todo]:
                f.result()
    if todo or _stale(LIB, objs) or _read(DIGEST_STAMP) != digest:
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs)
        with open(DIGEST_STAMP, "w") as f:
            f.write(digest + "\n")
    if verbose:
        print("built", LIB, "digest", digest)
    return LIB


def loaded_digest() -> str:
    """gs_build_digest() of the libgsplat_amd.so this process loads (ctypes on
    the in-tree file: the same object the torch binding links).  torch is
    imported first so the HIP runtime the library binds to is torch's own
    (libamdhip64.so.7 is resolved by soname: whichever loads first serves the
    process; a ctypes load ahead of torch would put /opt/rocm's runtime under
    torch -- under rocprofv3 --pmc no kernel of ours was dispatched then)."""
    import ctypes
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB)
    lib.gs_build_digest.restype = ctypes.c_char_p
    return lib.gs_build_digest().decode()


def check_loaded_digest() -> str:
    """Refuse a library built from other sources than the tree's: returns the
    digest when gs_build_digest() of the loaded library equals source_digest(),
    raises otherwise."""
    got, want = loaded_digest(), source_digest()
    if got != want:
        raise RuntimeError(f"libgsplat_amd.so was built from sources with digest {got}, the tree's is {want}: "
                           "rebuild (python gaussian_splatting_with_eye_tracking_amd/build.py)")
    return got


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    incs = ce.include_paths()
    libdirs = ce.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = ["-O2", "-std=c++17", "-fPIC", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", f"-I{sysconfig.get_paths()['include']}", "-I/opt/rocm/include", f"-I{INCLUDE}"]
    cflags += [f"-I{p}" for p in incs]
    ldflags = [f"-L{p}" for p in libdirs] + [f"-Wl,-rpath,{p}" for p in libdirs]
    ldflags += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
                "-L/opt/rocm/lib", "-lamdhip64", f"-L{PKG}", "-lgsplat_amd", "-Wl,-rpath,$ORIGIN"]
    return cflags, ldflags


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def build_torch_ext(verbose: bool = False) -> str:
    out = ext_path()
    src = os.path.join(CSRC, "torch_ext.cpp")
    if _stale(out, [src, LIB] + _headers()):
        cflags, ldflags = _torch_flags()
        cxx = os.environ.get("CXX", "g++")
        _run([cxx] + cflags + [src, "-o", out] + ldflags)
    if verbose:
        print("built", out)
    return out


def source_digest() -> str:
    """16-hex digest of everything the native library is built from (sources,
    headers, compiler flags).  Profiles record it so bench.py attaches counter
    summaries only to the build they were measured on."""
    import hashlib
    h = hashlib.sha256()
    files = [os.path.join(CSRC, s) for s in HIP_SOURCES] + sorted(_headers()) + [os.path.join(CSRC, "torch_ext.cpp")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(f for f in HIP_FLAGS if not f.startswith("-I")).encode())  # (paths differ per box)
    h.update(repr(sorted(SOURCE_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def build_all(verbose: bool = False) -> None:
    build_hip_lib(verbose=verbose)
    build_torch_ext(verbose=verbose)


if __name__ == "__main__":
    build_all(verbose=True)
    sys.exit(0)
