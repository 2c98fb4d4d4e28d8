"""MFMA hazard audit of a gfx950 device-assembly listing (developer tool).

python tools/hazard_audit.py <file.s> [--kernel SUBSTR] [-v] [--json OUT]

Builds each function's control-flow graph (basic blocks split at labels and branches, edges to the fall-through
and to every branch target) and measures, along EVERY path, the wait states between each v_mfma and the
instructions that interact with its registers.  A wait state is one instruction, N + 1 for `s_nop N`; the text of
inline asm (between ;;#ASMSTART / ;;#ASMEND) is counted as the instructions it holds, which is what the hardware
executes (hipcc's hazard recognizer does not look inside it).  Classes:

  valu_ab   VALU write of an MFMA's A/B register -> the MFMA (backward walk; a memory return ends it)
  valu_c    VALU write of an MFMA's C register -> the MFMA
  d_read    the MFMA's D registers read by a non-MFMA instruction (VALU, ds_write, global/scratch store, ...)
  d_write   the MFMA's D registers overwritten by a non-MFMA instruction (WAW)
  d_ab      the MFMA's D registers read as A/B by a later MFMA
  d_c_part  the MFMA's D registers read as C by a later MFMA whose C is not exactly this D (partial overlap)
  war_c     a non-MFMA instruction writing a register the MFMA reads as C while the MFMA may still read it
  war_ab    a VALU / v_mov writing a register the MFMA reads as A/B, fewer than --war-ab states after it
  spill_addr  a scratch reload whose destination is used as a memory address (listed, with the states between)

Required wait states (--req): the gfx940 rules of LLVM's GCNHazardRecognizer for an 8-pass XDL op
(v_mfma_f32_32x32x16_f16 on gfx950), each + 1 for gfx950, rounded up: valu_ab 2, valu_c 2, d_read 12, d_write 12,
d_ab 12, d_c_part 11, war_c 8.  war_ab has no published rule (the operands are read at issue); sites under 4 are
listed for inspection.  Exit status 1 when any site is below its requirement (--strict-min N: below N for valu_ab).
"""
import argparse, collections, json, re, sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
REQ = {"valu_ab": 2, "valu_c": 2, "d_read": 12, "d_write": 12, "d_ab": 12, "d_c_part": 11, "war_c": 8, "war_ab": 4}
HORIZON = 24   # states walked from each MFMA (every requirement is below it)


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


class Inst:
    __slots__ = ("line", "text", "op", "ops", "defs", "uses", "states", "asm")

    def __init__(self, line, text, asm):
        self.line, self.text, self.asm = line, text, asm
        self.op, rest = (text.split(None, 1) + [""])[:2]
        self.ops = split_ops(rest)
        self.states = int(self.ops[0]) + 1 if self.op == "s_nop" and self.ops else 1
        self.defs, self.uses = set(), set()
        op = self.op
        if op.startswith("s_") or not self.ops:
            return
        # stores and scratch/global/buffer/ds writes: no VGPR destination
        atomic = "atomic" in op or (op.startswith("ds_") and not op.startswith(("ds_read", "ds_write", "ds_swizzle",
                                                                                   "ds_bpermute", "ds_permute")))
        returns = ("rtn" in op) if op.startswith("ds_") else (" sc0" in self.text or " glc" in self.text)
        no_dst = "store" in op or op.startswith("ds_write") or (atomic and not returns)
        if no_dst:
            for o in self.ops:
                self.uses |= regs(o)
        else:
            self.defs = regs(self.ops[0])
            for o in self.ops[1:]:
                self.uses |= regs(o)
        if op.startswith("v_") and ("_sdwa" in op or "op_sel" in self.text) and not is_mfma(op):
            self.uses |= self.defs   # partial writes read the rest of the destination


def is_mfma(op):
    return op.startswith(("v_mfma", "v_smfmac"))


def is_valu(op):
    return op.startswith("v_") and not is_mfma(op)


def is_mem(op):
    return op.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_"))


class Func:
    def __init__(self, name):
        self.name = name
        self.insts = []          # Inst
        self.blocks = []         # [start, end) indices
        self.block_of = []
        self.succ = []
        self.pred = []
        self.label_block = {}

    def build(self, labels_at):
        starts = {0}
        for i, ins in enumerate(self.insts):
            if i in labels_at:
                starts.add(i)
            if ins.op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                starts.add(i + 1)
        starts = sorted(s for s in starts if s <= len(self.insts))
        self.blocks = [(s, e) for s, e in zip(starts, starts[1:] + [len(self.insts)]) if s < e]
        self.block_of = [0] * len(self.insts)
        for b, (s, e) in enumerate(self.blocks):
            for i in range(s, e):
                self.block_of[i] = b
        lab2blk = {}
        for i, names in labels_at.items():
            if i < len(self.insts):
                for n in names:
                    lab2blk[n] = self.block_of[i]
        self.succ = [[] for _ in self.blocks]
        for b, (s, e) in enumerate(self.blocks):
            last = self.insts[e - 1]
            if last.op.startswith(("s_branch", "s_cbranch")):
                tgt = last.ops[0] if last.ops else None
                if tgt in lab2blk:
                    self.succ[b].append(lab2blk[tgt])
            if not last.op.startswith(("s_branch", "s_endpgm", "s_setpc")) and b + 1 < len(self.blocks):
                self.succ[b].append(b + 1)
        self.pred = [[] for _ in self.blocks]
        for b, ss in enumerate(self.succ):
            for t in ss:
                self.pred[t].append(b)

    def walk_fwd(self, i):
        """yield (index, states between insts[i] and it) along every path, up to HORIZON states"""
        seen = {}
        stack = [(i + 1, 0)]
        while stack:
            j, ws = stack.pop()
            while True:
                if ws >= HORIZON:
                    break
                if j >= len(self.insts):
                    break
                b = self.block_of[j]
                s, e = self.blocks[b]
                if j == s:
                    if seen.get(j, 1 << 30) <= ws:
                        break
                    seen[j] = ws
                yield j, ws
                ws += self.insts[j].states
                if j + 1 < e:
                    j += 1
                    continue
                for t in self.succ[b][1:]:
                    stack.append((self.blocks[t][0], ws))
                if not self.succ[b]:
                    break
                j = self.blocks[self.succ[b][0]][0]

    def walk_bwd(self, i):
        """yield (index, states between it and insts[i]) along every path backwards"""
        seen = {}
        stack = [(i - 1, 0)]
        while stack:
            j, ws = stack.pop()
            while True:
                if ws >= HORIZON or j < 0:
                    break
                b = self.block_of[j]
                s, e = self.blocks[b]
                if j == e - 1:
                    if seen.get(j, 1 << 30) <= ws:
                        break
                    seen[j] = ws
                yield j, ws
                ws += self.insts[j].states
                if j > s:
                    j -= 1
                    continue
                ps = self.pred[b]
                for t in ps[1:]:
                    stack.append((self.blocks[t][1] - 1, ws))
                if not ps:
                    break
                j = self.blocks[ps[0]][1] - 1


def parse(path):
    funcs, f = [], None
    labels_at = collections.defaultdict(list)
    in_asm = False
    for ln, l in enumerate(open(path).read().split("\n"), 1):
        if ";;#ASMSTART" in l:
            in_asm = True
            continue
        if ";;#ASMEND" in l:
            in_asm = False
            continue
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s*(;.*)?$", l)
        if m and not m.group(1).startswith(".L"):
            if f is not None:
                f.build(labels_at)
            f = Func(m.group(1))
            funcs.append(f)
            labels_at = collections.defaultdict(list)
            continue
        if f is None:
            continue
        s = l.split(";")[0].strip()
        if not s:
            continue
        lm = re.match(r"^(\.LBB\w+):", s)
        if lm:
            labels_at[len(f.insts)].append(lm.group(1))
            continue
        if s.startswith(".") or s.endswith(":"):
            continue
        f.insts.append(Inst(ln, s, in_asm))
    if f is not None:
        f.build(labels_at)
    return funcs


def audit(funcs, ksub, req):
    sites = collections.defaultdict(list)   # class -> (func, line, states, producer text, consumer text)
    minima = collections.defaultdict(lambda: 1 << 30)
    counts = collections.Counter()
    for fn in funcs:
        if ksub and ksub not in fn.name:
            continue
        ins = fn.insts
        for i, m in enumerate(ins):
            if m.op.startswith("scratch_load"):
                dst = m.defs
                for j, ws in fn.walk_fwd(i):
                    x = ins[j]
                    if x.op.startswith("s_waitcnt"):
                        continue
                    addr = None
                    if x.op.startswith(("global_", "flat_", "buffer_")) and len(x.ops) >= 2:
                        addr = x.ops[0] if x.defs == set() else x.ops[1]
                    elif x.op.startswith("ds_") and x.ops:
                        addr = x.ops[0] if x.defs == set() else x.ops[1]
                    if addr is not None and regs(addr) & dst:
                        sites["spill_addr"].append((fn.name, x.line, ws, m.text, x.text))
                        break
                    if x.defs & dst:
                        break
            if not is_mfma(m.op) or len(m.ops) < 4:
                continue
            counts["mfma"] += 1
            D, A, B, C = (regs(o) for o in m.ops[:4])
            AB = A | B
            # --- backward: VALU writes of A/B/C
            left_ab, left_c = set(AB), set(C)
            for j, ws in fn.walk_bwd(i):
                x = ins[j]
                if not (left_ab or left_c):
                    break
                if is_valu(x.op) and x.defs:
                    hab, hc = x.defs & left_ab, x.defs & left_c
                    if hab:
                        _note(sites, minima, "valu_ab", ws, fn, x, m, req)
                    if hc:
                        _note(sites, minima, "valu_c", ws, fn, x, m, req)
                    left_ab -= hab
                    left_c -= hc
                elif is_mem(x.op) or is_mfma(x.op):
                    left_ab -= x.defs
                    left_c -= x.defs
            # --- forward: readers / writers of D, writers of A/B/C
            live_d = set(D)
            for j, ws in fn.walk_fwd(i):
                x = ins[j]
                if is_mfma(x.op) and len(x.ops) >= 4:
                    xd, xa, xb, xc = (regs(o) for o in x.ops[:4])
                    if (xa | xb) & live_d:
                        _note(sites, minima, "d_ab", ws, fn, m, x, req)
                    if xc & live_d and xc != D:
                        _note(sites, minima, "d_c_part", ws, fn, m, x, req)
                    if xc == D:
                        break   # the accumulate chain: the next MFMA owns these registers now
                    live_d -= xd
                    continue
                if x.uses & live_d:
                    _note(sites, minima, "d_read", ws, fn, m, x, req)
                if x.defs & live_d:
                    _note(sites, minima, "d_write", ws, fn, m, x, req)
                    live_d -= x.defs
                if is_valu(x.op) or x.op.startswith("v_"):
                    if x.defs & C and C != D:
                        _note(sites, minima, "war_c", ws, fn, m, x, req)
                    if x.defs & AB:
                        _note(sites, minima, "war_ab", ws, fn, m, x, req)
    return sites, minima, counts


def _note(sites, minima, cls, ws, fn, prod, cons, req):
    minima[cls] = min(minima[cls], ws)
    if ws < req[cls]:
        sites[cls].append((fn.name, cons.line, ws, prod.text, cons.text))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--strict-min", type=int, default=None,
                    help="valu_ab requirement (the operand-fence policy: 16)")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    req = dict(REQ)
    if a.strict_min is not None:
        req["valu_ab"] = a.strict_min
    funcs = parse(a.asm)
    sites, minima, counts = audit(funcs, a.kernel, req)
    bad = 0
    print(f"{counts['mfma']} MFMAs audited in {sum(1 for f in funcs if a.kernel in f.name)} functions")
    for cls in list(REQ) + ["spill_addr"]:
        s = sites.get(cls, [])
        hist = collections.Counter(x[2] for x in s)
        mn = minima.get(cls)
        mn = "-" if mn is None or mn >= 1 << 30 else mn
        flag = cls not in ("war_ab", "spill_addr")
        if flag:
            bad += len(s)
        print(f"  {cls:10s} req {req.get(cls, '-'):>2}  min seen {mn!s:>3}  sites below: {len(s):5d}  "
              f"{dict(sorted(hist.items()))}")
        if a.v:
            for fn, ln, w, prod, cons in s[:40]:
                print(f"      {ln}: ws={w}  {prod}  ->  {cons}")
    if a.json:
        json.dump({k: [list(x) for x in v] for k, v in sites.items()} | {"minima": dict(minima)},
                  open(a.json, "w"), indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
