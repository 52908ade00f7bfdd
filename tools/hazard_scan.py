"""Scan gfx950 assembly for the two inline-asm hazards the compiler does not pad (DESIGN.md
section 10, "Hazards found"): (1) a VALU write of a VGPR followed by a DPP instruction reading it
as src0 with fewer than 2 wait states in between; (2) the DPP FMAC (inline asm, the depthwise)
writing a VGPR followed by an MFMA reading it with fewer than 2 wait states in between (gfx940+:
LLVM GCNHazardRecognizer's LegacyVALUNotDotWritesVGPRWaitStates = 2).  A hit is a
pair at distance d <= 2 (d = 1: adjacent, d = 2: one instruction or an s_nop 0 between).  s_nop N
counts as N + 1 wait states, s_waitcnt as none (measured: an s_waitcnt as the only instruction
between the two gave wrong MFMA results, DESIGN.md sections 4.5, A.14).  Linear scan per function (labels do not reset the window).

usage: python tools/hazard_scan.py kernel.s [function-name-substring]
"""
import re
import sys

VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok):
    out = set()
    for m in VREG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(lines, want=None):
    fn, hits = None, []
    last_valu = {}   # vgpr -> (position, opcode)
    pos = 0
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":") and not s.startswith("."):
            if not s.startswith(".L"):
                fn, last_valu, pos = s[:-1], {}, 0
            continue
        if s.startswith(".") or (want and (fn is None or want not in fn)):
            continue
        parts = s.replace(",", " ").split()
        op = parts[0]
        if op.startswith("s_nop"):
            pos += int(parts[1], 0) + 1
            continue
        if op.startswith("s_waitcnt"):
            continue   # no wait state: an s_waitcnt alone between the depthwise and its MFMA broke k_update_rr
        if op.startswith("s_"):
            pos += 1
            continue
        ops = parts[1:]
        if op.startswith("v_") and ("row_shr" in s or "row_shl" in s or "quad_perm" in s or "row_ror" in s):
            src0 = regs(ops[1]) if len(ops) > 1 else set()
            for r in src0:
                if r in last_valu and pos - last_valu[r][0] <= 2:
                    hits.append((fn, "VALU->DPP src0 d=%d" % (pos - last_valu[r][0]), last_valu[r][1], s))
        if op.startswith("v_mfma"):
            srcs = set()
            for t in ops[1:3]:
                srcs |= regs(t)
            for r in srcs:
                if r in last_valu and last_valu[r][1].startswith("v_pk_fmac_f16_dpp") and pos - last_valu[r][0] <= 2:
                    hits.append((fn, "DPP-FMAC->MFMA d=%d" % (pos - last_valu[r][0]), last_valu[r][1], s))
        if op.startswith("v_") and not op.startswith("v_mfma") and ops:
            for r in regs(ops[0]):
                last_valu[r] = (pos, op)
        pos += 1
    return hits


if __name__ == "__main__":
    want = sys.argv[2] if len(sys.argv) > 2 else None
    hits = scan(open(sys.argv[1]).read().splitlines(), want)
    import collections
    kinds = collections.Counter(h[1] for h in hits)
    for h in hits[:40]:
        print(*h, sep=" | ")
    print(dict(kinds))
    print(f"{len(hits)} with fewer than 2 wait states")
    sys.exit(1 if hits else 0)
