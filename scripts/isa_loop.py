"""Per-loop instruction counts of one kernel in a hipcc -S dump: finds natural loops from the
'Loop Header' annotations and counts instruction classes between the header label and the back
edge.  python scripts/isa_loop.py dump.s kernel_substring"""
import collections
import re
import sys

text = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*:", l) and sys.argv[2] in l)
end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
body = text[start:end + 1]
headers = {}
for i, l in enumerate(body):
    m = re.search(r"Header=(BB\S+)", l)
    if m:
        headers.setdefault(m.group(1), []).append(i)
    m = re.match(r"^\.L(BB\S+):.*Loop Header", l)
    if m:
        headers.setdefault(m.group(1), []).append(i)
for h, idx in headers.items():
    lo, hi = min(idx), max(idx)
    # extend to the last instruction before the next label after hi
    j = hi + 1
    while j < len(body) and not re.match(r"^\.LBB", body[j]):
        j += 1
    seg = [l.strip() for l in body[lo:j]]
    ops = [l.split()[0] for l in seg if l and not l.startswith((";", ".")) and not l.endswith(":")]
    c = collections.Counter(ops)
    cls = collections.Counter()
    for op, n in c.items():
        cls["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_")
            else "vmem" if op.startswith(("global_", "buffer_")) else "other"] += n
    print(h, f"lines {lo}-{j}", dict(cls))
    for op in ("v_mov_b64_e32", "v_mov_b32_e32", "v_readlane_b32", "v_writelane_b32", "v_cndmask_b32_e64",
               "v_cndmask_b32_e32", "v_mad_u64_u32", "v_bitop3_b32", "v_fmac_f64_e32", "v_fma_f64", "s_barrier"):
        if c[op]:
            print(f"   {c[op]:5d} {op}")
