"""Static instruction counts per barrier-delimited phase of a generated fused kernel (gfx950 asm from
`hipcc --cuda-device-only -S`).  Each part's iteration loop is the code between its s_barriers; the
counts are per wave per iteration.  Usage: python tools/isa_phases.py kernel.s"""
import collections
import re
import sys

seg = collections.Counter()
segs = []
kinds = ("VALU", "SALU", "LDS", "VMEM", "WAIT", "NOP")
for line in open(sys.argv[1]):
    t = line.strip()
    if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op == "s_barrier":
        segs.append(seg)
        seg = collections.Counter()
        continue
    if op.startswith("v_"):
        seg["VALU"] += 1
        if op.startswith("v_mov"):
            seg["vmov"] += 1
    elif op.startswith("ds_"):
        seg["LDS"] += 1
    elif op.startswith(("buffer_", "global_")):
        seg["VMEM"] += 1
    elif op == "s_waitcnt":
        seg["WAIT"] += 1
    elif op == "s_nop":
        seg["NOP"] += 1
    elif op.startswith("s_"):
        seg["SALU"] += 1
segs.append(seg)
names = ["VN+wr0", "CN0", "rd0+wr1", "CN1", "rd1", "(next)"]
print("segment  " + "  ".join(f"{k:>6s}" for k in kinds + ("vmov",)))
for i, s in enumerate(segs):
    print(f"{i:3d} {names[i % 6] if i < len(segs) - 1 else 'tail':8s}" + "  ".join(f"{s[k]:6d}" for k in kinds + ("vmov",)))
