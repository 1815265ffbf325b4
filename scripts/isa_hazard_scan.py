"""Scan a gfx950 kernel's ISA for VALU reads of MFMA results and report the issue slots between the
MFMA and the first reader (s_nop N counts N+1; other instructions 1).  Straight-line only: the scan
resets at labels and branches."""
import re, sys
f, kern = sys.argv[1], sys.argv[2]
lines = open(f).read().split("\n")
s = next(i for i, l in enumerate(lines) if l.startswith(kern + ":"))
e = next(i for i in range(s, len(lines)) if "s_endpgm" in lines[i])
def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m: return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    if m: return {int(m.group(1))}
    return set()
pending = {}  # vgpr -> (line, slots since, opcode)
out = []
for i in range(s, e):
    l = lines[i].split(";")[0].strip()
    if not l:
        continue
    if l.endswith(":") or l.startswith("s_cbranch") or l.startswith("s_branch") or l.startswith("s_setpc"):
        pending = {}
        continue
    op = l.split()[0]
    args = [a.strip() for a in l[len(op):].split(",")]
    adv = 1
    if op == "s_nop":
        adv = int(args[0], 0) + 1
    # reads
    if op.startswith("v_") and not op.startswith("v_mfma"):
        for a in args[1:]:
            for r in regs(a.lstrip("-").split()[0] if a else ""):
                if r in pending:
                    ln, dist, mop = pending[r]
                    out.append((dist, i + 1, ln + 1, mop, op))
                    for rr in list(pending):
                        if pending[rr][0] == ln:
                            del pending[rr]
                    break
    for r in list(pending):
        ln, dist, mop = pending[r]
        pending[r] = (ln, dist + adv, mop)
    if op.startswith("v_mfma"):
        for r in regs(args[0]):
            pending[r] = (i, 0, op)
    elif op.startswith("v_") and args:
        for r in regs(args[0]):
            pending.pop(r, None)
out.sort()
from collections import Counter
c = Counter((d, m.split("_")[2] + m.split("_")[3], o) for d, _, _, m, o in out if d < 12)
for k, v in sorted(c.items()):
    print(k, v)
print("closest:", out[:8])
