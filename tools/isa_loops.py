#!/usr/bin/env python3
"""Instruction mix of every loop in the kernels of a gfx950 .s file (hipcc --save-temps):
python tools/isa_loops.py file.s [kernel-substring].  A loop = the span from a label to the
last branch back to it."""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
sub = sys.argv[2] if len(sys.argv) > 2 else ""
kern = None
body = {}
for ln in src:
    m = re.match(r"^(_Z\w+):", ln)
    if m:
        kern = m.group(1)
        body[kern] = []
        continue
    if kern is not None:
        body[kern].append(ln)
        if ln.strip().startswith(".Lfunc_end"):
            kern = None


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_mov") or op.startswith("v_accvgpr"):
        return "v_mov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_write"
    if op.startswith("global_load") or op.startswith("buffer_load"):
        return "vmem_load"
    if op.startswith("global_store") or op.startswith("buffer_store"):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


for k, lines in body.items():
    if sub not in k:
        continue
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", ln) or re.search(r"s_branch\s+(\.LBB\w+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    print(f"== {k}")
    for a, b in loops:
        c = Counter()
        for ln in lines[a:b + 1]:
            t = ln.strip()
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            c[cls(t.split()[0])] += 1
        print(f"  loop lines {a}-{b}: " + " ".join(f"{kk}={v}" for kk, v in sorted(c.items())))
