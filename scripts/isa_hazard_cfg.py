"""Path-aware scan of one gfx950 kernel's ISA (hipcc -S output, one function) for short distances
between a v_mfma and the instructions that touch its registers afterwards, over every control-flow
path (branches and fall-through), not only straight-line code.

Per (producer, consumer class) pair it prints the smallest distance in issue slots (s_nop N counts
N + 1, every other instruction 1) along any path, and the places where a pair comes closer than
the smallest distance the same pair has in straight-line code (where the compiler's own hazard
recognizer sets the wait states) -- a cross-block path the recognizer may have missed.  Edges taken
only with EXEC = 0 (s_cbranch_execz taken, s_cbranch_execnz not taken) are left out.
--all-producers adds VALU producers with the gfx950 rules of vector_rule() and scans every function.

    python scripts/isa_hazard_cfg.py kernel.s [max_slots]     (one function, per-pair report)
    python scripts/isa_hazard_cfg.py --all[-producers] a.s b.s  (every function; exit 1 on a short pair)
"""
import re
import sys
from collections import defaultdict


def regs(tok):
    tok = tok.strip().lstrip("-")
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)\b", tok)
    if m:
        return {int(m.group(1))}
    return set()


def parse(path):
    ins = []  # (op, args, label_targets, raw)
    labels = {}
    for raw in open(path).read().split("\n"):
        line = raw.split(";")[0].strip()
        if not line:
            continue
        if line.endswith(":"):
            labels[line[:-1]] = len(ins)
            continue
        if line.startswith(".") or line.startswith("_") or ":" in line.split()[0]:
            continue
        op = line.split()[0]
        rest = line[len(op):]
        args = [a.strip() for a in rest.split(",")] if rest.strip() else []
        ins.append((op, args, line))
    return ins, labels


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_permlane"):
        return "permlane"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
        return "readlane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    return None


def dst_src(op, args):
    """(written vgprs, read vgprs, srcC vgprs for mfma)"""
    cls = classify(op)
    if cls is None or not args:
        return set(), set(), set()
    if cls == "mfma":
        return regs(args[0]), regs(args[1]) | regs(args[2]), regs(args[3]) if len(args) > 3 else set()
    if cls == "lds":
        if op.startswith("ds_read") or op.startswith("ds_bpermute") or op.startswith("ds_permute"):
            return regs(args[0]), set().union(*[regs(a) for a in args[1:]]) if len(args) > 1 else set(), set()
        return set(), set().union(*[regs(a) for a in args]), set()
    if cls == "vmem":
        if "load" in op:
            return regs(args[0]), set().union(*[regs(a) for a in args[1:]]) if len(args) > 1 else set(), set()
        return set(), set().union(*[regs(a) for a in args]), set()
    if cls == "readlane":
        return set(), regs(args[1]) if len(args) > 1 else set(), set()
    if op.startswith("v_writelane"):
        return regs(args[0]), set(), set()
    if op.startswith("v_cmp") and not op.startswith("v_cmpx"):
        # vcc / sgpr destination: every vgpr operand is a read
        return set(), set().union(*[regs(a.split()[0]) for a in args if a]), set()
    if cls == "permlane":  # swap: both operands read and written
        r = set().union(*[regs(a) for a in args[:2]])
        return r, r, set()
    w = regs(args[0])
    rd = set().union(*[regs(a.split()[0]) for a in args[1:] if a])
    return w, rd, set()


ALL_PRODUCERS = False  # --all-producers: VALU / permlane producers too, not only MFMA


def main(path, max_slots=24):
    ins, labels = parse(path)
    best = pairs(ins, labels, max_slots)
    report(ins, best, path)


def pairs(ins, labels, max_slots):
    n = len(ins)
    # predecessors
    preds = defaultdict(list)
    for i, (op, args, raw) in enumerate(ins):
        if op == "s_endpgm":
            continue
        if op == "s_branch":
            preds[labels[args[0]]].append(i)
            continue
        # edges taken only with EXEC = 0 (the wave then writes no vector register) are left out
        if op.startswith("s_cbranch") and op != "s_cbranch_execz":
            preds[labels[args[0]]].append(i)
        if i + 1 < n and op != "s_cbranch_execnz":
            preds[i + 1].append(i)
    cost = [int(a[0], 0) + 1 if op == "s_nop" else 1 for op, a, _ in ins]
    info = [dst_src(op, a) for op, a, _ in ins]
    best = {}  # (mfma idx, consumer idx, kind) -> distance

    for i in range(n):
        op, args, raw = ins[i]
        w, rd, rc = info[i]
        cls = classify(op)
        if cls is None:
            continue
        # registers this instruction touches that an earlier mfma may still be writing / reading
        want = {}
        for r in rd:
            want[r] = "RAW"
        if cls == "mfma":
            for r in rc:
                want.setdefault(r, "RAW_C")
        for r in w:
            want.setdefault(r, "WAW")
        if not want:
            continue
        # backward search over paths: (instr index, slots so far, straight flag, regs still open)
        ps0 = preds[i]
        stack = [(p, 0, len(ps0) == 1 and not ins[p][0].startswith("s_cbranch") and ins[p][0] != "s_branch",
                  frozenset(want)) for p in ps0]
        seen = {}
        while stack:
            j, d, st, open_regs = stack.pop()
            if d > max_slots or not open_regs:
                continue
            key = (j, open_regs)
            if key in seen and seen[key] <= d:
                continue
            seen[key] = d
            jw, jr, jc = info[j]
            jop = ins[j][0]
            if ALL_PRODUCERS and classify(jop) in ("valu", "permlane"):
                # a vector producer: every read of what it wrote (VALU -> MFMA operand, -> permlane,
                # transcendental -> use, ...); the straight-line minima tell which pairs need waits
                for r in open_regs & jw:
                    if want[r] in ("RAW", "RAW_C"):
                        k = (j, i, want[r])
                        if k not in best or d < best[k][0]:
                            best[k] = (d, st)
            if classify(jop) == "mfma":
                hit = open_regs & jw
                for r in hit:
                    kind = want[r]
                    if kind == "RAW_C" and regs(ins[i][1][3]) == jw:
                        continue  # same-accumulator chain: the hardware forwards it
                    k = (j, i, kind)
                    if k not in best or d < best[k][0]:
                        best[k] = (d, st)
                # a WAR: this instruction writes what the mfma still reads as srcC
                if cls != "mfma":
                    for r in (w & jc):
                        k = (j, i, "WAR_C")
                        if k not in best or d < best[k][0]:
                            best[k] = (d, st)
                open_regs = open_regs - jw
            else:
                open_regs = open_regs - jw
            nd = d + cost[j]
            ps = preds[j]
            for p in ps:
                stack.append((p, nd, st and len(ps) == 1 and not ins[p][0].startswith("s_cbranch")
                              and ins[p][0] != "s_branch", open_regs))
    return best


def report(ins, best, path):
    n = len(ins)
    agg = defaultdict(list)
    for (j, i, kind), (d, st) in best.items():
        agg[(kind, classify(ins[i][0]))].append((d, st, j, i))
    print(f"{path}: {n} instructions")
    for key in sorted(agg):
        v = agg[key]
        s_min = min((d for d, st, _, _ in v if st), default=None)
        a_min = min(d for d, _, _, _ in v)
        print(f"  {key[0]:6s} -> {key[1]:9s}: min {a_min:3d} over all paths, {s_min} in straight-line code, "
              f"{len(v)} pairs")
        if s_min is not None:
            for d, st, j, i in sorted(v):
                if d < s_min:
                    print(f"      CLOSER  d={d}  mfma@{j}: {ins[j][2]}")
                    print(f"                     user@{i}: {ins[i][2]}")


def split_functions(path):
    """(name, text) per kernel/function of a hipcc -S file"""
    out, cur, name = [], None, None
    for line in open(path).read().split("\n"):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur, name = [line], m.group(1)
            continue
        if cur is not None:
            cur.append(line)
            if line.startswith(".Lfunc_end"):
                out.append((name, "\n".join(cur)))
                cur = None
    return out


TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def vector_rule(prod, cons):
    """wait states after a VALU write (the gfx950 rules hipcc applies; the straight-line code of this
    library keeps each of them): 2 before an MFMA or a v_permlane reads the register, 1 before
    v_readlane / v_readfirstlane reads it, 1 after a transcendental before any VALU use"""
    cc = classify(cons)
    if cc in ("mfma", "permlane"):
        return 2
    if cc == "readlane":
        return 1
    if prod.startswith(TRANS) and cc == "valu":
        return 1
    return 0


def scan_all(paths, max_slots=24):
    """every function of every file: the MFMA / consumer pairs that some path brings closer than the
    smallest distance the compiler keeps for the same (MFMA opcode, hazard, consumer class) in
    straight-line code anywhere in these files (its own wait-state rule for that pair)"""
    import tempfile
    funcs = []
    for path in paths:
        for name, text in split_functions(path):
            if "v_mfma" not in text and not ALL_PRODUCERS:
                continue
            with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
                f.write(text)
            ins, labels = parse(f.name)
            funcs.append((path, name, ins, pairs(ins, labels, max_slots)))
    rule = {}
    for _, _, ins, rows in funcs:
        for (j, i, kind), (d, st) in rows.items():
            k = (ins[j][0], kind, classify(ins[i][0]))
            if st:
                rule[k] = min(rule.get(k, 99), d)
    print("straight-line minima (the compiler's rule):")
    for k in sorted(rule):
        print(f"    {k[0]:28s} {k[1]:6s} -> {k[2]:9s} {rule[k]}")
    bad = 0
    for path, name, ins, rows in funcs:
        hits = []
        for (j, i, kind), (d, st) in rows.items():
            k = (ins[j][0], kind, classify(ins[i][0]))
            if classify(ins[j][0]) == "mfma" and (kind == "RAW_C" or classify(ins[i][0]) == "mfma"):
                continue  # MFMA -> MFMA: the matrix core's own dependency checks
            if classify(ins[j][0]) == "mfma":
                need = rule.get(k, rule.get((ins[j][0], kind, "valu"), 0))
            else:
                need = vector_rule(ins[j][0], ins[i][0])
            if d < need:
                hits.append((d, need, kind, j, i))
        print(f"{path}: {name[:100]}: {len(hits)} short pairs")
        for d, need, kind, j, i in sorted(hits)[:12]:
            print(f"    {kind:5s} d={d} (<{need}) @{j}->{i}: {ins[j][2]}  ->  {ins[i][2]}")
        bad += len(hits)
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "--all-producers":
        ALL_PRODUCERS = True
        sys.argv[1] = "--all"
    if sys.argv[1] == "--all":
        sys.exit(1 if scan_all(sys.argv[2:]) else 0)
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 24)
