"""Native build driver: compiles every HIP/C++ source of the framework for gfx950.

No hipify, no CUDA shims: the kernels in ``csrc/kernels/*.hip`` are written for
CDNA4 directly and are compiled with ``hipcc --offload-arch=gfx950``.  The torch
binding layer (``csrc/bindings.cpp``) and the host runtime (``csrc/runtime/*.cpp``)
are compiled with the same toolchain and linked into ONE in-tree extension
``distributeddeeplearningspark_amd/_C.so`` (git-ignored, but it travels to the
GPU box with the gpurun snapshot).

Incremental: an object is rebuilt only when its source, any header under
``csrc/include`` or the compile flags changed.

Usage: ``python -m distributeddeeplearningspark_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import subprocess
import sys
import sysconfig
import time
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
OUT = PKG / "_C.so"
ARCH = os.environ.get("DDL_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (import only for its install location)
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(ce.__file__), "..", "lib")
    return inc, os.path.abspath(lib)


def _common_flags():
    return [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-munsafe-fp-atomics",
        "-I", str(CSRC / "include"),
        "-Wno-unused-result",
        "-Wno-unused-command-line-argument",
        *os.environ.get("DDL_HIPCC_FLAGS", "").split(),  # experiments, e.g. -DDDL_DMA_MIN_BLOCKS=4
    ]


# Per-kernel-file flags.  attention.hip: no SLP vectorisation (it packs the softmax row sums and the
# O rescale into v_pk_add/v_pk_mul_f32, which cost 20+ cycles each beside MFMAs on gfx950) and no NaN
# semantics for fmaxf (drops a canonicalising v_max per MFMA output in the running row maximum).
_FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize", "-fno-honor-nans"]}


def _binding_flags():
    import pybind11
    import torch

    inc, _ = _torch_paths()
    flags = []
    for p in inc:
        flags += ["-isystem", p]
    flags += ["-isystem", sysconfig.get_paths()["include"], "-isystem", pybind11.get_include()]
    flags += [
        f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-Wno-deprecated-declarations",
        "-Wno-ignored-attributes",
    ]
    return flags


def _sources():
    kern = sorted((CSRC / "kernels").glob("*.hip"))
    rt = sorted((CSRC / "runtime").glob("*.cpp"))
    binding = sorted(CSRC.glob("*.cpp"))
    return kern, rt, binding


def _hdr_digest():
    h = hashlib.sha1()
    for p in sorted((CSRC / "include").rglob("*")):
        if p.is_file():
            h.update(p.name.encode())
            h.update(p.read_bytes())
    return h.hexdigest()


def _obj_path(src: Path) -> Path:
    rel = src.relative_to(CSRC)
    return BUILD / (str(rel).replace(os.sep, "__") + ".o")


def _compile(src: Path, flags, hdr_digest: str, force: bool):
    obj = _obj_path(src)
    stamp = obj.with_suffix(".stamp")
    key = hashlib.sha1((src.read_bytes().decode("utf-8", "replace") + "\0".join(flags) + hdr_digest).encode()).hexdigest()
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == key:
        return obj, False, 0.0
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src.name}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    stamp.write_text(key)
    return obj, True, time.time() - t0


def build(jobs: int | None = None, force: bool = False, verbose: bool = True) -> Path:
    """Compile all native sources and link ``_C.so``. Returns the output path."""
    kern, rt, binding = _sources()
    hdr = _hdr_digest()
    base = _common_flags()
    bflags = base + _binding_flags()
    tasks = [(s, base + _FILE_FLAGS.get(s.name, [])) for s in kern] + [(s, bflags) for s in rt] + [(s, bflags) for s in binding]
    jobs = jobs or int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
    objs, rebuilt = [], False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(_compile, s, f, hdr, force): s for s, f in tasks}
        for fut in cf.as_completed(futs):
            obj, did, dt = fut.result()
            objs.append(obj)
            rebuilt |= did
            if did and verbose:
                print(f"[ddl-build] {futs[fut].name} ({dt:.1f}s)", flush=True)
    objs.sort()
    if not rebuilt and OUT.exists() and OUT.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return OUT
    _, tlib = _torch_paths()
    tmp = OUT.with_name(OUT.name + ".tmp")  # link aside, then an atomic rename: a reader never sees half a library
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
            f"-L{tlib}", f"-Wl,-rpath,{tlib}",
            "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip", "-ltorch_python",
            f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lrocprofiler-sdk-roctx",
            "-lpthread"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, OUT)
    if verbose:
        print(f"[ddl-build] linked {OUT} ({len(objs)} objects)", flush=True)
    (BUILD / "manifest.json").write_text(json.dumps({"arch": ARCH, "objects": [o.name for o in objs]}, indent=1))
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(a.jobs, a.force)


if __name__ == "__main__":
    sys.exit(main())
