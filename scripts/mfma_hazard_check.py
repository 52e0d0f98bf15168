#!/usr/bin/env python3
"""Flag inline-asm VALU reads of MFMA results that lack the wait states the hardware needs.

The compiler's hazard recognizer inserts the wait states between an XDL (MFMA) write of a VGPR
and a later VALU read of it, but it does not see into inline asm. The FP4 kernels' epilogues read
the accumulators with an inline-asm ``v_bfi_b32``; this walks the device assembly in straight-line
order (basic blocks as written, which is how the compiler lays out the epilogues) and reports every
``v_bfi_b32`` reading a VGPR that an MFMA wrote fewer than ``--wait`` issue slots before (each
instruction one slot, ``s_nop N`` N + 1). It is a lint on the emitted code, run after a build:

    hipcc --offload-arch=gfx950 -O3 -S --offload-device-only -Icsrc/include X.hip -o X.s
    python scripts/mfma_hazard_check.py X.s
"""
from __future__ import annotations

import argparse
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text: str) -> set[int]:
    out: set[int] = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(path: str, wait: int) -> list[str]:
    bad = []
    func = "?"
    recent: list[tuple[int, set[int]]] = []  # (slot at issue, written VGPRs)
    slot = 0
    for line in open(path):
        s = line.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":") and not s.startswith("."):
            if not s.startswith(".L"):
                func = s[:-1]
                recent.clear()
            continue
        if s.startswith("."):
            continue
        op, _, args = s.partition(" ")
        if op == "s_nop":
            slot += int(args.strip(), 0) + 1
            continue
        slot += 1
        if "mfma" in op:
            dst = args.split(",")[0]
            recent.append((slot, regs(dst)))
            recent = recent[-64:]
            continue
        if op == "v_bfi_b32":
            srcs = regs(",".join(args.split(",")[1:]))
            for at, w in recent:
                if srcs & w and slot - at < wait:
                    bad.append(f"{func[:90]}: '{s}' reads v{sorted(srcs & w)} {slot - at} slots after an MFMA wrote it")
                    break
    return bad


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("asm", nargs="+")
    ap.add_argument("--wait", type=int, default=19, help="issue slots required after a 16-pass XDL write")
    a = ap.parse_args()
    bad = [b for p in a.asm for b in check(p, a.wait)]
    for b in bad[:50]:
        print(b)
    print(f"{len(bad)} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
