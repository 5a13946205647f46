"""Instruction-class breakdown of the loops of one kernel in a hipcc -S listing (gfx950).

usage: python tools/isa_loops.py kernels.s _Z6k_walkILi7ELi2048EEv9walk_args
A loop is a label that some later branch in the function jumps back to; its body is the lines from
the label to that branch.  Classes: VALU by opcode family, SALU, SMEM, VMEM (global/buffer), LDS,
waits, branches, scratch (spill) traffic."""
import re
import sys
from collections import Counter


def body(lines, fn):
    start = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def klass(op: str) -> str:
    if op.startswith("v_mad_u64_u32"):
        return "v_mad_u64_u32"
    if op.startswith(("v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_subrev_co_u32",
                      "v_subbrev_co_u32")):
        return "v_add/sub carry"
    if op.startswith(("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add3_u32", "v_lshl_add_u32", "v_add_lshl_u32")):
        return "v_add/sub u32 (no carry)"
    if op.startswith(("v_mov_b32", "v_mov_b64", "v_pk_mov_b32")):
        return "v_mov"
    if op.startswith("v_cndmask"):
        return "v_cndmask"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "v_cmp"
    if op.startswith(("v_bitop3", "v_and", "v_or", "v_xor", "v_not", "v_bfi", "v_and_or", "v_or3", "v_xad", "v_xor3")):
        return "v_logic"
    if op.startswith(("v_lshl", "v_lshr", "v_ashr", "v_alignbit", "v_alignbyte", "v_bfe", "v_perm")):
        return "v_shift/perm"
    if op.startswith(("v_mul_", "v_mad_u32", "v_mul_hi", "v_mul_lo")):
        return "v_mul32"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "v_lane"
    if op.startswith("v_"):
        return "v_other:" + op
    if op.startswith(("scratch_", "buffer_store", "buffer_load")) and "off" in op:
        return "scratch"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other:" + op


def main():
    lines = open(sys.argv[1]).read().split("\n")
    fn = sys.argv[2]
    b = body(lines, fn)
    labels = {}
    for i, l in enumerate(b):
        m = re.match(r"^(\.LBB[0-9_]+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(b):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB[0-9_]+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    for s, e in loops:
        c = Counter()
        for l in b[s:e + 1]:
            t = l.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            c[klass(t.split()[0])] += 1
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"loop {b[s].split(':')[0]} lines {s}-{e}: {sum(c.values())} instructions, VALU {valu}")
        for k, v in sorted(c.items(), key=lambda x: -x[1]):
            print(f"  {v:6d}  {k}")


if __name__ == "__main__":
    main()
