"""ISA check of the streaming kernel's counted asm side-operand loads (residual rows, their ReLU mask, the BN
input x and its mask byte): along every control-flow path from such a load, no instruction reads or writes the
load's destination registers before an s_waitcnt whose vmcnt is at most the number of VMEM operations issued
after that load (the compiler does not know the loads are asynchronous, and with the one-tile-ahead prefetch the
wait sits in the next loop iteration).  Branch targets come from the instruction addresses in the disassembly.
Usage: python scripts/r6/check_side_loads.py (repo root, after the build)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributeddeeplearningspark_amd.utils.isa import code_objects  # noqa: E402

KERNELS = ["ILi16ELi256ELi1ELb1ELi1E", "ILi16ELi256ELi0ELb1ELi1E", "ILi16ELi256ELi1ELb0ELi2E", "ILi16ELi256ELi0ELb0ELi2E",
           "ILi16ELi256ELi1ELb0ELi1E", "ILi16ELi256ELi1ELb1ELi0E", "ILi32ELi256ELi1ELb1ELi0E", "ILi16ELi64ELi1ELb1ELi1E",
           "ILi32ELi64ELi1ELb1ELi1E", "ILi16ELi128ELi1ELb1ELi1E", "ILi32ELi128ELi1ELb1ELi1E", "ILi32ELi64ELi1ELb0ELi2E",
           "ILi32ELi128ELi1ELb0ELi2E", "ILi32ELi64ELi1ELb1ELi0E", "ILi64ELi64ELi1ELb1ELi0E", "ILi32ELi128ELi1ELb1ELi0E",
           "ILi16ELi128ELi1ELb1ELi0E", "ILi32ELi64ELi0ELb1ELi1E"]
_LOAD = re.compile(r"\s*global_load_(?:ushort|ubyte|dwordx2|dwordx4|dword)\s+(v\[\d+:\d+\]|v\d+),")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")


def _regs(tok):
    tok = tok.split("//")[0]
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
        text.append(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", f.name], capture_output=True,
                                   text=True).stdout)
        os.unlink(f.name)
    return "\n".join(text)


def _succ(lines, addr_of, idx_of, i):
    ins = lines[i].split("//")[0].strip()
    op = ins.split()[0] if ins else ""
    if op == "s_endpgm":
        return []
    if op.startswith("s_branch") or op.startswith("s_cbranch"):
        imm = int(ins.split()[-1])
        imm = imm - 65536 if imm >= 32768 else imm
        tgt = idx_of.get(addr_of[i] + 4 + 4 * imm)
        nxt = [tgt] if tgt is not None else []
        return nxt if op.startswith("s_branch") else nxt + [i + 1]
    return [i + 1]


def hazards(so=os.path.join(ROOT, "distributeddeeplearningspark_amd", "_C.so")):
    """[(kernel, load, instruction)] of register uses reachable before a covering wait."""
    dis = _disasm(so)
    found = []
    for name in KERNELS:
        m = re.search(r"\n[0-9a-f]+ <(_ZN3ddl18gemm_stream_kernel" + name + r"[^>]*)>:\n(.*?)(?=\n\n|\Z)", dis, re.S)
        if not m:
            raise LookupError(name)
        lines = [l for l in m.group(2).split("\n") if _ADDR.search(l)]
        addr_of = [int(_ADDR.search(l).group(1), 16) for l in lines]
        idx_of = {a: i for i, a in enumerate(addr_of)}
        first = min(i for i, l in enumerate(lines) if "global_load_lds" in l)
        for i in range(first, len(lines)):
            lm = _LOAD.match(lines[i].split("//")[0])
            if not lm:
                continue
            rs = _regs(lm.group(1))
            stack, seen = [(j, 0) for j in _succ(lines, addr_of, idx_of, i)], set()
            while stack:
                j, younger = stack.pop()
                if j >= len(lines) or (j, younger) in seen:
                    continue
                seen.add((j, younger))
                ins = lines[j].split("//")[0]
                w = re.search(r"s_waitcnt\s+vmcnt\((\d+)\)", ins)
                if w and int(w.group(1)) <= younger:
                    continue
                if rs & _regs(ins):
                    found.append((name, lines[i].split("//")[0].strip(), ins.strip()))
                    break
                y = min(64, younger + (1 if re.match(r"\s*(global_|buffer_)", ins) else 0))
                stack.extend((k, y) for k in _succ(lines, addr_of, idx_of, j))
    return found


if __name__ == "__main__":
    bad = hazards()
    for b in bad[:20]:
        print("HAZARD", *b)
    print(f"{len(KERNELS)} kernels checked, {len(bad)} hazards")
    sys.exit(1 if bad else 0)
