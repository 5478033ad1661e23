"""Instruction histogram of one kernel in a hipcc -S device assembly dump (static counts per loop
region, for VALU-budget work).  python scripts/isa_hist.py dump.s kernel_substring"""
import collections
import re
import sys

text = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*:", l) and name in l)
end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
body = [l.strip() for l in text[start:end + 1]]
ops = [l.split()[0] for l in body if l and not l.startswith((";", ".")) and not l.endswith(":")]
cnt = collections.Counter(ops)
cls = collections.Counter()
for op, n in cnt.items():
    k = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else \
        "vmem" if op.startswith(("global_", "buffer_")) else "other"
    cls[k] += n
print(dict(cls))
for op, n in cnt.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
    print(f"{n:5d} {op}")
