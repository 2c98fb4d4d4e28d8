"""VALU -> MFMA operand hazard audit of a gfx950 assembly listing (developer tool).

python tools/hazard_audit.py <file.s> [--min N] [--kernel SUBSTR]

For every v_mfma in every function, walks back through the instruction stream to the nearest VALU
instruction that writes one of the MFMA's A or B source registers and counts the wait states between them
(one per instruction, N + 1 per `s_nop N`).  Round 4 found that hipcc's 2 wait states after a
v_cvt_pk_f16_f32 that writes a B fragment are not always enough on MI355X (rare, timing-dependent stale
operands); this lists every site below --min (default 4) so each one can be padded.

The walk is linear: across a label it continues into the fall-through predecessor and marks the site
'label' (a branch predecessor may be closer); it stops after 64 instructions.
"""
import argparse, collections, re, sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((kind, r))
    return out


def split_ops(rest):
    # operands separated by commas outside brackets
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def is_valu(op):
    if not op.startswith("v_") or op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return False
    return not op.startswith(("v_cmp", "v_readfirstlane", "v_readlane"))  # these write SGPRs / VCC


def audit(path, min_ws, ksub):
    lines = open(path).read().split("\n")
    func = None
    insts = []  # (func, lineno, text)
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s*(;.*)?$", l)
        if m and not l.startswith(".") and not m.group(1).startswith(".L"):
            func = m.group(1)
            continue
        s = l.split(";")[0].strip()
        if not s:
            continue
        if re.match(r"^\.LBB\d+_\d+:", s):
            insts.append((func, i, "LABEL"))
            continue
        if s.startswith("."):
            continue
        insts.append((func, i, s))
    sites = []
    for idx, (fn, ln, s) in enumerate(insts):
        if not s.startswith("v_mfma") or (ksub and ksub not in (fn or "")):
            continue
        op, rest = (s.split(None, 1) + [""])[:2]
        ops = split_ops(rest)
        if len(ops) < 4:
            continue
        srcab = regs(ops[1]) | regs(ops[2])
        ws, crossed = 0, False
        j = idx - 1
        found = None
        steps = 0
        while j >= 0 and insts[j][0] == fn and steps < 64:
            t = insts[j][2]
            steps += 1
            if t == "LABEL":
                crossed = True
                j -= 1
                continue
            top, trest = (t.split(None, 1) + [""])[:2]
            if top.startswith("s_branch") or top == "s_endpgm":
                break  # not a fall-through predecessor
            if is_valu(top):
                tops = split_ops(trest)
                if tops and (regs(tops[0]) & srcab):
                    found = (t, ws)
                    break
            elif "load" in top or top.startswith("ds_read"):
                tops = split_ops(trest)
                hit = regs(tops[0]) & srcab if tops else set()
                srcab -= hit  # the latest write of these registers is a memory return, not a VALU
                if not srcab:
                    break
            if top == "s_nop":
                ws += int(trest.strip() or 0) + 1
            else:
                ws += 1
            j -= 1
        if found and found[1] < min_ws:
            sites.append((fn, ln + 1, found[1], found[0], s, crossed))
    return sites


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--min", type=int, default=4)
    ap.add_argument("--kernel", default="")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    sites = audit(a.asm, a.min, a.kernel)
    per = collections.Counter(s[0] for s in sites)
    hist = collections.Counter(s[2] for s in sites)
    print(f"{len(sites)} MFMA A/B operands written by VALU < {a.min} wait states before; by wait states: "
          f"{dict(sorted(hist.items()))}")
    for fn, n in per.most_common():
        print(f"  {n:5d}  {fn}")
    if a.v:
        for fn, ln, w, prod, cons, crossed in sites:
            print(f"{ln}: ws={w}{' (label)' if crossed else ''}  {prod}  ->  {cons}")
    return 1 if sites else 0


if __name__ == "__main__":
    sys.exit(main())
