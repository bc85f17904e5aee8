#!/usr/bin/env python3
"""Per-kernel device ISA of a libmirsha build, addresses stripped, for checking that
a source change leaves a kernel's code untouched (e.g. a diagnostic hook that must
compile to nothing in the product build):

    python3 tools/kernel_isa.py LIB.so [NAME_SUBSTRING] > isa.txt   # then diff two builds
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_dpp_hazards import disassemble  # noqa: E402


def kernels(so):
    out, cur = {}, None
    for line in disassemble(so):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m and re.match(r"^L\d+$", m.group(1)):  # a branch target inside the kernel
            if cur:
                out[cur].append(m.group(1) + ":")
            continue
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and line.strip():
            ins = line.split("//")[0].strip()
            ins = re.sub(r"\b0x[0-9a-f]+\b", "X", ins) if ins.startswith("s_cbranch") or ins.startswith("s_branch") else ins
            out[cur].append(ins)
    return out


def normalized(ins):
    """Label names renumbered per kernel in order of appearance (llvm-objdump numbers
    them across the whole file, so adding a kernel renames every later label)."""
    names = {}

    def sub(m):
        return names.setdefault(m.group(0), "L%d" % len(names))
    return [re.sub(r"\bL\d+\b", sub, x) for x in ins]


if __name__ == "__main__":
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, ins in sorted(kernels(sys.argv[1]).items()):
        if sub in name:
            print("==", name, len(ins))
            print("\n".join(normalized(ins)))
