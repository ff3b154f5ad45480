"""Inspect the gfx950 machine code inside the built extension (no GPU needed).

``_C.so`` carries one clang offload bundle per HIP translation unit in its ``.hip_fatbin``
section; each bundle holds the gfx950 code object (an AMDGPU ELF).  This module extracts
them, disassembles with ``llvm-objdump`` and tallies instructions per kernel, so tests and
reports can check *statically* that the hot kernels really issue MFMA instructions, use
the LDS transpose reads / direct-to-LDS loads, and never spill to scratch.  (``rocprofv3 --pmc SQ_INSTS_MFMA...`` gives the dynamic counterpart.)
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile
from collections import Counter

LLVM = os.environ.get("DDL_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path: str, name: str = ".hip_fatbin") -> bytes:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sec.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section={name}={out}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        with open(out, "rb") as f:
            return f.read()


def code_objects(path: str, arch: str = "gfx950") -> list[bytes]:
    """Every ``hipv4-amdgcn-amd-amdhsa--<arch>`` code object in the extension's fat binary."""
    blob = _section(path)
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24 : q + 24 + tlen].decode()
            q += 24 + tlen
            if triple.endswith(arch) and size:
                out.append(blob[pos + off : pos + off + size])
        pos = blob.find(MAGIC, pos + len(MAGIC))
    return out


_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def kernel_instruction_counts(path: str, arch: str = "gfx950", loop_scratch: dict | None = None) -> dict[str, Counter]:
    """{mangled kernel symbol: Counter(mnemonic)} over all code objects.  ``loop_scratch`` (optional dict) receives
    {symbol: scratch instructions placed before the kernel's LAST s_barrier} — for the LDS-staged GEMM / conv
    kernels, whose K-loop ends at its last barrier, the spills that the main loop can execute."""
    res: dict[str, Counter] = {}
    order: dict[str, list] = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(path, arch)):
            f = os.path.join(d, f"co{i}.o")
            with open(f, "wb") as fh:
                fh.write(co)
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", f"--mcpu={arch}", f],
                                 check=True, capture_output=True, text=True).stdout
            cur = None
            for line in dis.splitlines():
                m = _FUNC.match(line.strip())
                if m:
                    cur = res.setdefault(m.group(1), Counter())
                    seq = order.setdefault(m.group(1), [])
                    continue
                s = line.strip()
                if cur is None or not s or s.startswith(";") or ":" in s.split()[0]:
                    continue
                cur[s.split()[0]] += 1
                if loop_scratch is not None and (s.startswith("scratch_") or s.startswith("s_barrier")):
                    seq.append(s.split()[0])
    if loop_scratch is not None:
        for k, seq in order.items():
            last = max((i for i, op in enumerate(seq) if op == "s_barrier"), default=-1)
            loop_scratch[k] = sum(1 for op in seq[:last] if op.startswith("scratch_"))
    return res


def demangle(names):
    for tool in (os.path.join(LLVM, "llvm-cxxfilt"), "c++filt"):
        try:
            r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True)
            out = r.stdout.splitlines()
            if len(out) == len(names):
                return out
        except Exception:
            continue
    return list(names)


def summary(path: str, arch: str = "gfx950") -> list[dict]:
    """Per-kernel rows: MFMA / LDS-transpose / LDS-DMA / scratch instruction counts."""
    loop = {}
    counts = kernel_instruction_counts(path, arch, loop)
    names = list(counts)
    rows = []
    for name, pretty in zip(names, demangle(names)):
        c = counts[name]
        tot = sum(c.values())
        rows.append({
            "kernel": pretty,
            "instructions": tot,
            "mfma": sum(v for k, v in c.items() if k.startswith("v_mfma")),
            "ds_read_tr": sum(v for k, v in c.items() if k.startswith("ds_read_b64_tr")),
            "lds_dma": sum(v for k, v in c.items() if k.startswith(("buffer_load", "global_load_lds"))
                           and "lds" in k),
            "scratch": sum(v for k, v in c.items() if k.startswith("scratch_")),
            "loop_scratch": loop.get(name, 0),
        })
    rows.sort(key=lambda r: -r["mfma"])
    return rows
