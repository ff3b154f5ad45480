"""ISA check of the streaming kernel's counted asm side-operand loads (residual rows,
their ReLU mask, the BN input x and its mask byte): no instruction reads or writes a load's destination
registers between the load and the first s_waitcnt after the tile barrier whose vmcnt is at most the number of
VMEM operations issued after that load (the compiler does not know the loads are asynchronous).  Usage: python scripts/r6/check_side_loads.py (repo root, after the build)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributeddeeplearningspark_amd.utils.isa import code_objects  # noqa: E402

KERNELS = [(k, 0) for k in ("ILi16ELi256ELi1ELb1ELi1E", "ILi16ELi256ELi0ELb1ELi1E", "ILi16ELi256ELi1ELb0ELi2E",
                            "ILi16ELi256ELi1ELb0ELi1E", "ILi16ELi256ELi1ELb1ELi0E", "ILi32ELi256ELi1ELb1ELi0E",
                            "ILi16ELi64ELi1ELb1ELi1E", "ILi32ELi64ELi1ELb1ELi1E", "ILi16ELi128ELi1ELb1ELi1E",
                            "ILi32ELi128ELi1ELb1ELi1E", "ILi32ELi64ELi1ELb0ELi2E", "ILi32ELi128ELi1ELb0ELi2E",
                            "ILi32ELi64ELi1ELb1ELi0E", "ILi64ELi64ELi1ELb1ELi0E", "ILi32ELi128ELi1ELb1ELi0E",
                            "ILi16ELi128ELi1ELb1ELi0E", "ILi32ELi64ELi0ELb1ELi1E", "ILi16ELi256ELi0ELb0ELi2E")]
_LOAD = re.compile(r"\s*global_load_(?:ushort|ubyte|dwordx2|dwordx4|dword)\s+(v\[\d+:\d+\]|v\d+),")


def _regs(tok):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", tok):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"(?<![\[:\d])v(\d+)\b", tok):
        out.add(int(m.group(1)))
    return out


def _disasm(so):
    text = []
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".o", delete=False) as f:
            f.write(co)
        text.append(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", f.name],
                                   capture_output=True, text=True).stdout)
        os.unlink(f.name)
    return "\n".join(text)


def hazards(so=os.path.join(ROOT, "distributeddeeplearningspark_amd", "_C.so")):
    """[(kernel, line)] of register uses before the counted wait; raises if a listed kernel is missing."""
    dis = _disasm(so)
    found = []
    for name, D in KERNELS:
        m = re.search(r"\n[0-9a-f]+ <(_ZN3ddl18gemm_stream_kernel" + name + r"[^>]*)>:\n(.*?)(?=\n\n|\Z)", dis, re.S)
        if not m:
            raise LookupError(name)
        lines = m.group(2).split("\n")
        first = min(i for i, l in enumerate(lines) if "global_load_lds" in l)
        for i in range(first, len(lines)):
            lm = _LOAD.match(lines[i])
            if not lm:
                continue
            rs, barrier, younger = _regs(lm.group(1)), False, 0
            for j in range(i + 1, len(lines)):
                if "s_barrier" in lines[j]:
                    barrier = True
                w = re.search(r"s_waitcnt vmcnt\((\d+)\)", lines[j])
                if barrier and w and int(w.group(1)) <= younger:  # vmcnt(k) with k <= later VMEM ops: done
                    break
                if rs & _regs(lines[j]):
                    found.append((name, lines[j].strip()))
                    break
                if re.match(r"\s*(global_|buffer_)", lines[j]):
                    younger += 1
    return found


if __name__ == "__main__":
    bad = hazards()
    for b in bad:
        print("HAZARD", *b)
    print(f"{len(KERNELS)} kernels checked, {len(bad)} hazards")
    sys.exit(1 if bad else 0)
