#!/usr/bin/env python3
"""Instruction mix of one kernel's hottest loop in a hipcc -S assembly file.

Usage: isa_mix.py FILE.s SYMBOL-SUBSTRING
Finds the kernel, picks the loop whose back edge spans the most instructions
(the row loop of the step kernels), and counts its instructions by class.
Tuning aid only; nothing in the product imports it.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sym):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and sym in l.split(":")[0]:
            start = i
            continue
        if start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel not found: " + sym)


def classify(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_mov_b64") or op.startswith("v_mov_b32") or op.startswith("v_accvgpr"):
        return "valu_mov"
    if op.startswith("v_cndmask"):
        return "valu_select"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("global_load") or op.startswith("buffer_load"):
        return "vmem_load"
    if op.startswith("global_store") or op.startswith("buffer_store"):
        return "vmem_store"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_"):
        return "salu/branch"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, sym)
    labels = {}
    ins = []  # (index, op, text)
    for l in body:
        s = l.strip()
        m = re.match(r"^(\.L\w+):", s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        ins.append((op, s))
    best = None
    for i, (op, s) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                span = i - labels[tgt]
                if best is None or span > best[1]:
                    best = (labels[tgt], span, tgt)
    print("kernel instructions:", len(ins))
    if best is None:
        print("no loop")
        return
    lo, span, tgt = best
    c = Counter(classify(op) for op, _ in ins[lo : lo + span + 1])
    f64 = Counter(op for op, _ in ins[lo : lo + span + 1] if classify(op) == "valu_f64")
    oth = Counter(op for op, _ in ins[lo : lo + span + 1] if classify(op) in ("valu_other", "valu_mov", "valu_select"))
    print("loop", tgt, "instructions:", span + 1)
    for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
        print("  %-14s %5d" % (k, v))
    print("  f64 ops:", dict(f64.most_common()))
    print("  other valu:", dict(oth.most_common(20)))


if __name__ == "__main__":
    main()
