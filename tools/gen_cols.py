#!/usr/bin/env python3
"""Generate keyhunt_amd/csrc/kh_cols.h: the product-scanning columns of fe_mul / fe_sqr as one asm
statement per column, scheduled so that no s_nop is needed inside a column.

Why (profiles/r03b_ubench_cost.txt): on gfx950 a VALU instruction that reads an SGPR
lane mask written by an earlier VALU instruction (the carry of v_mad_u64_u32, read as carry-in by
the v_addc_co_u32 that counts it) needs wait states; emitted as one asm statement per product, hipcc
pads every multiply-add and every count with an s_nop (fe_mul: ~115 per multiplication).  At 4
waves/SIMD those pads cost: 16 multiply-adds + 16 counts take 63 SIMD cycles with them and 46 when
each count reads a mask written >= 2 instructions earlier.

Column k holds the products p = 0..n-1 (a_i * b_j, i + j = k).  Each product is one
`v_mad_u64_u32 acc, m, a, b, acc` whose 65th bit lands in the SGPR pair m; every product after the
first `safe` ones (which provably cannot carry) is counted by `v_addc_co_u32 cnt, m, 0, cnt, m`
(carry-out written back into the mask it read: a write-after-write on an SGPR needs no wait state,
the listing holds such pairs).  Masks rotate over three SGPR pairs and every count is emitted at
least GAP instructions after its multiply-add, with an s_nop only where a short column has nothing
else to place there.  The accumulator chain itself (VGPR read-after-write) is interlocked by the
hardware.  The scheduler below asserts both rules for every column it emits.

usage: python tools/gen_cols.py > keyhunt_amd/csrc/kh_cols.h
"""
GAP = 2  # independent instructions (or s_nop wait states) between a mask's write and its read


def schedule(n: int, safe: int):
    """Order of ('mad', p) / ('cnt', p) / ('nop', w) for a column of n products, the first `safe`
    of them uncounted; masks m[p % 3]."""
    out = []
    pending = []  # counted products whose count is not yet emitted, in order
    pos = {}      # instruction index of each product's multiply-add

    def waited(q):  # wait states since product q's multiply-add (an s_nop w gives w + 1)
        return sum(x[1] + 1 if x[0] == "nop" else 1 for x in out[pos[q] + 1:])
    for p in range(n):
        # emit ready counts first while keeping at most 2 masks outstanding before a third mad
        while pending and len(pending) >= 2:
            q = pending[0]
            if waited(q) < GAP:
                break
            out.append(("cnt", q))
            pending.pop(0)
        if len(pending) >= 3:
            raise AssertionError("mask reuse before read")
        pos[p] = len(out)
        out.append(("mad", p))
        if p >= safe:
            pending.append(p)
        # a count becomes due once GAP instructions follow its mad
        if len(pending) >= 2:
            q = pending[0]
            if waited(q) >= GAP:
                out.append(("cnt", q))
                pending.pop(0)
    while pending:
        q = pending[0]
        gap = waited(q)
        if gap < GAP:
            out.append(("nop", GAP - gap - 1))  # s_nop w = w + 1 wait states
            continue
        out.append(("cnt", q))
        pending.pop(0)
    check(out, n, safe)
    return out


def check(out, n, safe):
    """Every count reads its own mask >= GAP wait states after the mad wrote it, and no mad rewrote
    that mask in between."""
    waits = []
    for ins in out:
        waits.append(ins[1] + 1 if ins[0] == "nop" else 1)
    for idx, ins in enumerate(out):
        if ins[0] != "cnt":
            continue
        p = ins[1]
        mi = next(i for i, x in enumerate(out) if x == ("mad", p))
        assert sum(waits[mi + 1:idx]) >= GAP, (n, safe, out)
        for x in out[mi + 1:idx]:
            assert not (x[0] == "mad" and x[1] % 3 == p % 3), (n, safe, out)
    assert sorted(x[1] for x in out if x[0] == "mad") == list(range(n))
    assert sorted(x[1] for x in out if x[0] == "cnt") == list(range(safe, n))


def col_asm(n: int, safe: int, first_zero: bool):
    """asm text: %0 acc (in/out 64-bit, or out only when first_zero: the column starts from 0),
    %1 cnt (out), %2..%4 masks, product p's operands at %(5+2p), %(6+2p)."""
    lines = []
    counted = 0
    for ins in schedule(n, safe):
        if ins[0] == "mad":
            p = ins[1]
            src2 = "0" if (first_zero and p == 0) else "%0"
            lines.append(f"v_mad_u64_u32 %0, %{2 + p % 3}, %{5 + 2 * p}, %{6 + 2 * p}, {src2}")
        elif ins[0] == "cnt":
            m = f"%{2 + ins[1] % 3}"
            prev = "%1" if counted else "0"
            lines.append(f"v_addc_co_u32 %1, {m}, 0, {prev}, {m}")
            counted += 1
        else:
            lines.append(f"s_nop {ins[1]}")
    return "\\n\\t".join(lines), counted


def emit_column(name_acc: str, prods: list[tuple[str, str]], safe: int, first_zero: bool, indent="  "):
    n = len(prods)
    text, counted = col_asm(n, safe, first_zero)
    ins = ", ".join(f'"v"({a}), "v"({b})' for a, b in prods)
    acc_c = f'"=&v"({name_acc})' if first_zero else f'"+v"({name_acc})'
    cnt_c = '"=&v"(cnt)' if counted else '"=&v"(cnt_unused)'
    return (f'{indent}asm("{text}"\n{indent}    : {acc_c}, {cnt_c}, "=&s"(m0), "=&s"(m1), "=&s"(m2)\n'
            f'{indent}    : {ins});\n'), counted


def gen():
    out = ['// kh_cols.h -- GENERATED by tools/gen_cols.py: the product-scanning columns of fe_mul and',
           '// fe_sqr, one asm statement per column, scheduled so that every carry count reads a mask',
           '// written >= 2 instructions earlier (no s_nop inside a column).  See the generator.',
           '// Included by kh_math.h inside namespace kh (device compilation only).',
           '#pragma once', '', '#if defined(__HIP_DEVICE_COMPILE__)', '']
    # fe_mul: t = a * b (16 limbs)
    out.append('// t[0..15] = a * b')
    out.append('__device__ __forceinline__ void mul_cols(const uint32_t *a, const uint32_t *b, uint32_t t[16]) {')
    out.append('  uint64_t acc, m0, m1, m2;')
    out.append('  uint32_t cnt, cnt_unused;')
    for k in range(15):
        prods = [(f"a[{i}]", f"b[{k - i}]") for i in range(8) if 0 <= k - i <= 7]
        # column 0 and the first product of column 1 cannot carry: (2^32-1)^2 + 2^32 - 1 < 2^64
        safe = len(prods) if k == 0 else (1 if k == 1 else 0)
        s, counted = emit_column("acc", prods, safe, k == 0)
        out.append(s.rstrip("\n"))
        out.append(f"  t[{k}] = (uint32_t)acc;")
        hi = "((uint64_t)cnt << 32)" if counted else "0"
        out.append(f"  acc = (acc >> 32) | {hi};")
    out.append("  t[15] = (uint32_t)acc;")
    out.append("  (void)cnt_unused;")
    out.append("}")
    out.append("")
    # fe_sqr cross products a_i * a_j, i < j: columns 1..13 (t[0] = 0, t[14..15] from the last acc)
    out.append('// t[1..15] = sum_{i<j} a_i a_j 2^(32(i+j)) (t[0] = 0): the cross products of a square, not doubled')
    out.append('__device__ __forceinline__ void sqr_cross_cols(const uint32_t *a, uint32_t t[16]) {')
    out.append('  uint64_t acc, m0, m1, m2;')
    out.append('  uint32_t cnt, cnt_unused;')
    out.append('  t[0] = 0;')
    for k in range(1, 14):
        prods = [(f"a[{i}]", f"a[{k - i}]") for i in range(8) if i < k - i <= 7]
        # columns 1 and 2 hold one cross product each and column 3 starts on an accumulator of at
        # most 2^32 - 1: their first products cannot carry
        safe = 1 if k <= 3 else 0
        s, counted = emit_column("acc", prods, safe, k == 1)
        out.append(s.rstrip("\n"))
        out.append(f"  t[{k}] = (uint32_t)acc;")
        hi = "((uint64_t)cnt << 32)" if counted else "0"
        out.append(f"  acc = (acc >> 32) | {hi};")
    out.append("  t[14] = (uint32_t)acc;")
    out.append("  t[15] = (uint32_t)(acc >> 32);")
    out.append("  (void)cnt_unused;")
    out.append("}")
    out += ["#endif"]
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(gen(), end="")
