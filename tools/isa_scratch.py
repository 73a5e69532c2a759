#!/usr/bin/env python3
"""Where a kernel's scratch (spill) accesses sit: registers, spill counts and every scratch_* instruction with
the loop depth of its basic block, from the device assembly of one source file.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include --offload-device-only -S \\
        csrc/src/hip/tile16_kernels.hip -o build/tile16.s
    python tools/isa_scratch.py build/tile16.s tile16_slide_kernel

Depth 0 is the kernel body outside any loop; LLVM annotates each block inside a loop nest with its depth
("in Loop: Header=... Depth=N"), so a spill at depth d runs once per iteration of the d-th enclosing loop.
"""
import collections
import re
import sys


def functions(asm, pattern):
    for m in re.finditer(r"^(_Z\S*" + re.escape(pattern) + r"\S*):", asm, re.M):
        name = m.group(1)
        end = asm.index(".Lfunc_end", m.end())
        yield name, asm[m.end():end]


def metadata(asm, name):
    i = asm.find(".name:           " + name)
    if i < 0:
        i = asm.find(".name: " + name)
    block = asm[max(0, i - 2500):i + 2500] if i >= 0 else ""
    out = {}
    for key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
        m = re.search(r"\." + key + r":\s+(\d+)", asm[i:i + 3000]) if i >= 0 else None
        out[key] = int(m.group(1)) if m else None
    return out


def main():
    if len(sys.argv) < 3:
        print(__doc__)
        return 2
    asm = open(sys.argv[1]).read()
    for name, body in functions(asm, sys.argv[2]):
        lines = body.split("\n")
        depth = 0
        hits = []
        for line in lines:
            if line.startswith(".LBB") or line.startswith("; %bb"):
                m = re.search(r"Depth=(\d+)", line)
                depth = int(m.group(1)) if m else 0
            if "scratch_" in line and not line.strip().startswith(";"):
                hits.append((depth, line.strip()))
        print(name)
        print("  ", metadata(asm, name))
        print("   scratch accesses by loop depth:", dict(sorted(collections.Counter(d for d, _ in hits).items())))
        for d, ins in hits:
            print(f"     depth {d}: {ins}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
