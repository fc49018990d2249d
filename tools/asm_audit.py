#!/usr/bin/env python3
"""Audit the gfx950 assembly of inline-asm MFMA kernels (hipcc -save-temps .s file).

For every kernel whose name matches: register counts, spills / scratch, and the compiler's own
accumulator traffic between the first and the last MFMA (v_accvgpr_mov / _read / _write outside
;;#ASMSTART / ;;#ASMEND blocks). With accumulators held as "a" operands of asm MFMAs, hipcc
pads no XDL-write -> read wait states around them: any compiler v_accvgpr_* inside the MFMA
region is a potential silent corruption and must be zero (cdna_hip_programming.md §5.7 item 4).
usage: asm_audit.py FILE.s [NAME_SUBSTR]"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):(?:\s*;.*)?$", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())  # (a kernel can have several s_endpgm)
        yield name, text[m.end():end]


def meta(text, name):
    i = text.find(".name:           " + name)
    if i < 0:
        i = text.find(name, text.find("amdhsa.kernels"))
    lo = text.rfind("\n  - ", 0, i)
    hi = text.find("\n  - ", i)
    blk = text[lo:hi if hi > 0 else len(text)]
    out = {}
    for key in ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
        mm = re.search(r"\." + key + r":\s+(\d+)", blk)
        out[key] = int(mm.group(1)) if mm else None
    return out


def _regs(tok):
    """set of (kind, index) for a register operand like v[4:7], v12, a[0:3]"""
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def valu_to_mfma(lines):
    """VALU (or v_accvgpr_write) results read as an A/B operand by an MFMA within the next 2
    instructions: the hazard needs 2 wait states, which hipcc does not pad for asm MFMAs."""
    real = []
    for l in lines:
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        real.append(t)
    bad = []
    for i, t in enumerate(real):
        if not t.startswith("v_mfma"):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        srcs = _regs(ops[1]) | _regs(ops[2])
        nops = 0
        for back in range(1, 4):
            if i - back < 0:
                break
            u = real[i - back]
            if u.startswith("s_nop"):
                nops += int(u.split()[1]) + 1
                continue
            if nops >= 2 or back - 1 + nops >= 2:
                break
            if u.startswith("v_") and not u.startswith("v_mfma") and not u.startswith("v_cmp"):
                dst = u.split(None, 1)[1].split(",")[0].strip() if " " in u else ""
                if _regs(dst) & srcs:
                    bad.append(u + "  ->  " + t)
    return bad


def mfma_d_to_reader(lines, states=12):
    """Non-MFMA instructions that touch a VGPR MFMA result within `states` wait states of the
    MFMA (8-pass XDL: 12), counting s_nop N as N + 1 states and other instructions as 1."""
    real = []
    for l in lines:
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        real.append(t)
    bad = []
    for i, t in enumerate(real):
        if not t.startswith("v_mfma"):
            continue
        dst = _regs(t.split(None, 1)[1].split(",")[0].strip())
        if not dst or next(iter(dst))[0] != "v":
            continue
        n = 0
        for u in real[i + 1:i + 1 + states]:
            if n >= states:
                break
            if u.startswith("s_nop"):
                n += int(u.split()[1]) + 1
                continue
            if u.startswith("v_mfma"):
                ops = [o.strip() for o in u.split(None, 1)[1].split(",")]
                if _regs(ops[3]) == dst:
                    break  # accumulate chain: no wait states
            regs = set()
            for tok in re.split(r"[\s,]+", u.split(None, 1)[1] if " " in u else ""):
                regs |= _regs(tok)
            if regs & dst:
                bad.append(t + "  ->  " + u)
                break
            n += 1
    return bad


def audit(body):
    lines = body.splitlines()
    # the region the AGPR accumulators are live in: first .. last MFMA writing an AGPR
    idx = [i for i, l in enumerate(lines) if "v_mfma" in l and l.split(None, 1)[1].lstrip().startswith("a")]
    if not idx:
        idx = [i for i, l in enumerate(lines) if "v_mfma" in l]
    if not idx:
        return {"mfma": 0}
    lo, hi = idx[0], idx[-1]
    inasm = False
    bad = []
    scratch = 0
    for i, l in enumerate(lines):
        if ";;#ASMSTART" in l:
            inasm = True
        elif ";;#ASMEND" in l:
            inasm = False
        elif lo <= i <= hi and not inasm and "v_accvgpr" in l:
            bad.append(l.strip())
        if lo <= i <= hi and "scratch_" in l:
            scratch += 1
    haz = valu_to_mfma(lines) + mfma_d_to_reader(lines)
    return {"mfma": sum("v_mfma" in l for l in lines), "compiler_accvgpr_in_mfma_region": len(bad), "scratch_ops_in_mfma_region": scratch,
            "valu_to_mfma_hazards": len(haz), "examples": bad[:3] + haz[:3]}


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    ok = True
    for name, body in kernels(text):
        if sub not in name:
            continue
        m, a = meta(text, name), audit(body)
        print(name[:90], m, {k: v for k, v in a.items() if k != "examples"})
        for e in a.get("examples", []):
            print("    ", e)
        if a.get("compiler_accvgpr_in_mfma_region") or a.get("valu_to_mfma_hazards") or (m.get("vgpr_spill_count") or 0):
            ok = False
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
