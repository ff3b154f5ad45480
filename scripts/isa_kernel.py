"""Dump one kernel's gfx950 disassembly from the built extension and summarise its main loop.
Usage: python scripts/isa_kernel.py <mangled-name-substring> [out.s]"""
import collections
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributeddeeplearningspark_amd.utils.isa import code_objects  # noqa: E402

LL = "/opt/rocm/lib/llvm/bin"
want = sys.argv[1]
for co in code_objects("distributeddeeplearningspark_amd/_C.so"):
    with tempfile.NamedTemporaryFile(suffix=".o", delete=False) as f:
        f.write(co)
        fn = f.name
    out = subprocess.run([f"{LL}/llvm-objdump", "-d", "--no-show-raw-insn", fn], capture_output=True, text=True).stdout
    for m in re.finditer(r"\n[0-9a-f]+ <([^>]*)>:\n(.*?)(?=\n\n|\Z)", out, re.S):
        if want not in m.group(1):
            continue
        lines = [l.split("//")[0].strip() for l in m.group(2).splitlines() if l.strip()]
        ops = collections.Counter(l.split()[0] for l in lines)
        print(m.group(1), len(lines), "instr")
        print({k: ops[k] for k in ops if any(t in k for t in ("mfma", "global_load", "ds_read", "s_waitcnt", "scratch", "s_barrier", "buffer"))})
        waits = [l for l in lines if l.startswith("s_waitcnt") and "vmcnt" in l]
        print("vmcnt waits:", collections.Counter(waits).most_common(8))
        if len(sys.argv) > 2:
            open(sys.argv[2], "w").write("\n".join(lines))
        sys.exit(0)
print("not found")
