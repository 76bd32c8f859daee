"""Packed-FP32 forwarding pairs in a gfx950 device assembly file (hipcc --cuda-device-only -S).

A *pair* is a v_pk_{add,mul,fma}_f32 (the producer) immediately followed by an instruction that
reads one of the producer's destination VGPRs.  The compiler puts one `s_nop 0` between such a
pair exactly when the producer's first source has op_sel_hi = 1 (the default): LLVM's
dst-sel-forwarding check reads bit 3 of src0_modifiers, which on VOP3 is DST_OP_SEL and on VOP3P
is op_sel_hi[0].  Producers written with op_sel_hi[0] = 0 (the PLL mixer's
`v_pk_mul_f32 v[24:25], v[6:7], v[24:25] op_sel:[0,1] op_sel_hi:[0,0]`) therefore get no wait
state.  Round 6 tests whether that missing wait state is the configs[3] chain fault
(c.re = x.re * v.re in lanes 48-63 when bank MFMA waves share the PLL wave's SIMD).

  python tools/diag/pk_hazard_edit.py report IN.s              per-kernel pair census
  python tools/diag/pk_hazard_edit.py MODE IN.s OUT.s          write an edited copy
MODE: rt (unchanged), after12 (s_nop 0 after every uncovered producer whose consumer reads it as
src1/src2), before12 (the same count of s_nop 0 placed BEFORE those producers: timing control),
after0 (s_nop 0 after uncovered producers read only as src0), all4 (s_nop 4 after EVERY
v_pk_{add,mul,fma}_f32, covered or not: the widest wait state).  Diagnostic only.
"""
import re
import sys
from collections import Counter, defaultdict

PK = re.compile(r"^\s*(v_pk_(?:add|mul|fma)_f32)\s")


def vregs(tok):
    tok = tok.strip().lstrip("-|").rstrip("|")
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def operands(line):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    ops = [o.strip() for o in parts[1].split(",")]
    if ops:  # trailing modifiers ride on the last operand: "v[2:3] op_sel_hi:[0,1]"
        ops[-1] = ops[-1].split()[0] if ops[-1] else ops[-1]
    return parts[0], ops


def opsel_hi0(line):
    m = re.search(r"op_sel_hi:\[(\d)", line)
    return 1 if m is None else int(m.group(1))


def is_insn(line):
    s = line.strip()
    return bool(s) and not s.startswith((";", ".")) and not s.endswith(":") and not s.startswith("//")


def pairs(lines):
    """(index of producer, slot class '12' or '0', covered?, kernel) for every pair."""
    out = []
    insn = [i for i, l in enumerate(lines) if is_insn(l)]
    for a, b in zip(insn, insn[1:]):
        la = lines[a]
        m = PK.match(la)
        if not m:
            continue
        _, pops = operands(la)
        if not pops:
            continue
        dst = vregs(pops[0])
        lb = lines[b]
        covered = lb.strip().startswith("s_nop")
        if covered:  # the consumer is the instruction after the nop
            nxt = [j for j in insn if j > b][:1]
            if not nxt:
                continue
            lb = lines[nxt[0]]
        bop, bops = operands(lb)
        if not bop.startswith("v_") or not bops:
            continue
        slots = [k for k, o in enumerate(bops[1:]) if vregs(o) & dst]
        if not slots:
            continue
        out.append((a, "12" if any(k >= 1 for k in slots) else "0", covered, opsel_hi0(la)))
    return out


def kernel_of(lines):
    names, cur = [], None
    for l in lines:
        m = re.match(r"^(_Z\S*):", l)
        if m:
            cur = m.group(1)
        names.append(cur)
    return names


def main():
    mode, src = sys.argv[1], sys.argv[2]
    lines = open(src).read().split("\n")
    ps = pairs(lines)
    if mode == "report":
        kn = kernel_of(lines)
        census = defaultdict(Counter)
        for a, cls, cov, oh in ps:
            census[kn[a]][(cls, "covered" if cov else "UNCOVERED")] += 1
        for k in sorted(census):
            c = census[k]
            print(f"{c[('12', 'UNCOVERED')]:5d} {c[('0', 'UNCOVERED')]:5d} {c[('12', 'covered')]:5d} "
                  f"{c[('0', 'covered')]:5d}  {k}")
        print("columns: uncovered src1/2, uncovered src0, covered src1/2, covered src0")
        # the compiler's rule, checked: covered <=> op_sel_hi[0] == 1
        rule = Counter((cov, oh) for _, _, cov, oh in ps)
        print("(covered, op_sel_hi[0]) counts:", dict(rule))
        return
    dst = sys.argv[3]
    sel = {"after12": ("12", "after"), "before12": ("12", "before"), "after0": ("0", "after")}
    edits = {}
    if mode in sel:
        cls, where = sel[mode]
        for a, c, cov, _ in ps:
            if c == cls and not cov:
                edits[a] = where
    nop = "\ts_nop 0"
    if mode == "all4":
        edits = {i: "after" for i, l in enumerate(lines) if PK.match(l)}
        nop = "\ts_nop 4"
    out = []
    for i, l in enumerate(lines):
        if edits.get(i) == "before":
            out.append(nop)
        out.append(l)
        if edits.get(i) == "after":
            out.append(nop)
    open(dst, "w").write("\n".join(out))
    print(f"{mode}: {len(edits)} {nop.strip()} inserted", file=sys.stderr)


if __name__ == "__main__":
    main()
