#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc ``-S`` listing (gfx950).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --cuda-device-only \
        -S -o /tmp/fedagg.s flame_amd/csrc/fedagg.hip -Iinclude
    python tools/isa_count.py /tmp/fedagg.s fedopt_chain_kernelILi1ELi0ELi8E [--block LABEL] [--top 40]

Prints the opcode histogram of the function whose label contains the pattern (or of one basic
block of it, ``--block .LBB12_7``: the loop body a PMC count divides by), grouped into VALU /
SALU / VMEM / LDS / branch classes.  DESIGN.md §4's per-element-step counts come from this plus
``rocprofv3 --pmc SQ_INSTS_VALU`` on the same build.
"""
import argparse
import collections
import re
import sys


def body(lines, pattern):
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^[_A-Za-z0-9.$]+:", ln) and pattern in ln.split(":")[0]:
            start = i
            continue
        if start is not None and (ln.startswith(".Lfunc_end") or re.match(r"^\s*\.size\s", ln)):
            return lines[start:i]
    if start is None:
        sys.exit(f"no function label contains {pattern!r}")
    return lines[start:]


def blocks(fn):
    out, cur, name = collections.OrderedDict(), [], "entry"
    for ln in fn:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            out[name] = cur
            name, cur = m.group(1), []
            continue
        cur.append(ln)
        if re.match(r"^\s*s_cbranch", ln):        # a conditional branch ends a block too (fallthrough: name+)
            out[name] = cur
            name, cur = name + "+", []
    out[name] = cur
    return out


def opcodes(lines):
    ops = []
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        ops.append(s.split()[0])
    return ops


def klass(op):
    if op.startswith(("v_mfma", "v_smfmac")):
        return "MFMA"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep")):
        return "wait/nop"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("pattern")
    ap.add_argument("--block", default=None, help="one basic block (label) instead of the whole function")
    ap.add_argument("--blocks", action="store_true", help="list the function's blocks with their sizes")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    fn = body(open(a.listing).read().splitlines(), a.pattern)
    bl = blocks(fn)
    if a.blocks:
        for nm, b in bl.items():
            ops = opcodes(b)
            c = collections.Counter(klass(o) for o in ops)
            print(f"{nm:14s} {len(ops):5d} ops  " + "  ".join(f"{k} {v}" for k, v in c.most_common()))
        return
    ops = opcodes(bl[a.block] if a.block else fn)
    by = collections.Counter(klass(o) for o in ops)
    print(f"{len(ops)} instructions: " + ", ".join(f"{k} {v}" for k, v in by.most_common()))
    for op, n in collections.Counter(ops).most_common(a.top):
        print(f"  {n:6d}  {op}  [{klass(op)}]")


if __name__ == "__main__":
    main()
