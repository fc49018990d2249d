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
        end = text.find("s_endpgm", m.end())
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


def audit(body):
    lines = body.splitlines()
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
    return {"mfma": len(idx), "compiler_accvgpr_in_mfma_region": len(bad), "scratch_ops_in_mfma_region": scratch,
            "examples": bad[:3]}


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
        if a.get("compiler_accvgpr_in_mfma_region") or (m.get("vgpr_spill_count") or 0):
            ok = False
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
