"""VGPR / AGPR / LDS / scratch of the kernels whose symbol contains a substring (code-object metadata of _C.so).
Usage: python scripts/r6/vgpr.py <substring> [...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributeddeeplearningspark_amd.utils.isa import code_objects  # noqa: E402

with tempfile.TemporaryDirectory() as d:
    for i, co in enumerate(code_objects(os.path.join(ROOT, "distributeddeeplearningspark_amd", "_C.so"))):
        fn = os.path.join(d, f"co{i}.o")
        open(fn, "wb").write(co)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", fn], capture_output=True, text=True).stdout
        for blk in re.split(r"\n\s+- \.", out):
            m = re.search(r"\.name:\s+(\S+)", blk)
            if not m or not any(w in m.group(1) for w in sys.argv[1:]):
                continue
            g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "-"])[1]
            print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>3} lds {g('group_segment_fixed_size'):>6} "
                  f"scratch {g('private_segment_fixed_size'):>4}  {m.group(1)[:90]}")
