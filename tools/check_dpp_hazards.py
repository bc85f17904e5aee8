#!/usr/bin/env python3
"""Check the built gfx950 code object for the VALU -> DPP read hazard.

CDNA3/4 need 2 wait states between a VALU instruction that writes a VGPR and a
DPP instruction whose lane-crossing source (src0) reads it. LLVM's hazard
recognizer inserts the s_nop for DPP it generates itself, but not for DPP inside
inline asm (k_digest_chain2's MSHA_DROUND): there the asm text carries its own
s_nop. This script disassembles libmirsha.so's device code and, for every *_dpp
instruction, walks back 2 wait states (an instruction is one, s_nop N is N + 1)
and fails if any VALU instruction in that window writes the DPP's src0, or if
the window crosses a branch target (then the predecessor is not known).

    python3 tools/check_dpp_hazards.py [libmirsha.so]      # exit 1 on a hazard

Used by tests/test_abi.py::test_no_dpp_read_hazard_in_device_code.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WAIT_STATES = 2
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def _regs(tok: str) -> set:
    m = _VREG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def disassemble(so: str) -> list:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                       capture_output=True)
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", "--mcpu=gfx950", co],
                             check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def check(lines: list) -> tuple[int, list]:
    """(number of DPP instructions, list of hazard descriptions)."""
    insts = []   # (kind, mnemonic, operands, text); kind "i" instruction, "L" label / function start
    for ln in lines:
        s = ln.split("//")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            insts.append(("L", "", [], s))
            continue
        parts = s.split(None, 1)
        mnem = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        insts.append(("i", mnem, ops, s))
    n_dpp, bad = 0, []
    for k, (kind, mnem, ops, text) in enumerate(insts):
        if kind != "i" or not mnem.endswith("_dpp") or len(ops) < 2:
            continue
        n_dpp += 1
        src0 = _regs(ops[1].split()[0])
        waits, j = 0, k - 1
        while waits < WAIT_STATES:
            if j < 0 or insts[j][0] == "L":
                bad.append(f"{text}: branch target or function start within {WAIT_STATES} wait states")
                break
            _, m2, o2, t2 = insts[j]
            if m2 == "s_nop":
                waits += int(o2[0], 0) + 1 if o2 else 1
            else:
                if m2.startswith("v_") and o2 and _regs(o2[0]) & src0:
                    bad.append(f"{text}: src0 written {waits} wait state(s) earlier by '{t2}'")
                    break
                waits += 1
            j -= 1
    return n_dpp, bad


def main() -> int:
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mirbft_amd", "libmirsha.so")
    n, bad = check(disassemble(so))
    for b in bad:
        print("HAZARD", b)
    print(f"{n} DPP instructions checked, {len(bad)} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
