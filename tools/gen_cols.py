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
NM = 4   # SGPR pairs the masks rotate over: up to NM - 1 counts outstanding, so a column's last
         # counts need no pad (3 pairs left one s_nop at the end of most columns)


def schedule(n: int, safe: int):
    """Order of ('mad', p) / ('cnt', p) / ('nop', w) for a column of n products, the first `safe`
    of them uncounted; masks m[p % NM]."""
    out = []
    pending = []  # counted products whose count is not yet emitted, in order
    pos = {}      # instruction index of each product's multiply-add

    def waited(q):  # wait states since product q's multiply-add (an s_nop w gives w + 1)
        return sum(x[1] + 1 if x[0] == "nop" else 1 for x in out[pos[q] + 1:])
    for p in range(n):
        # emit ready counts first while keeping at most 2 masks outstanding before a third mad
        while pending and len(pending) >= NM - 1:
            q = pending[0]
            if waited(q) < GAP:
                break
            out.append(("cnt", q))
            pending.pop(0)
        if len(pending) >= NM:
            raise AssertionError("mask reuse before read")
        pos[p] = len(out)
        out.append(("mad", p))
        if p >= safe:
            pending.append(p)
        # a count becomes due once GAP instructions follow its mad
        if len(pending) >= NM - 1:
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
            assert not (x[0] == "mad" and x[1] % NM == p % NM), (n, safe, out)
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
            lines.append(f"v_mad_u64_u32 %0, %{2 + p % NM}, %{2 + NM + 2 * p}, %{3 + NM + 2 * p}, {src2}")
        elif ins[0] == "cnt":
            m = f"%{2 + ins[1] % NM}"
            prev = "%1" if counted else "0"
            lines.append(f"v_addc_co_u32 %1, {m}, 0, {prev}, {m}")
            counted += 1
        else:
            lines.append(f"s_nop {ins[1]}")
    return "\\n\\t".join(lines), counted


def emit_column(name_acc: str, prods: list[tuple[str, str]], safe: int, first_zero: bool, indent="  ",
                shift_in: bool = False):
    """shift_in: the previous column counted no carry, so this column's accumulator is the previous
    one shifted down 32 bits -- one v_lshrrev_b64 at the head of the statement (the C form
    `acc >> 32` compiles to a move pair through a zero register)."""
    n = len(prods)
    text, counted = col_asm(n, safe, first_zero)
    if shift_in:  # from a separate input (the previous accumulator keeps its low word, a t limb)
        text = f"v_lshrrev_b64 %0, 32, %{2 + NM + 2 * n}\\n\\t" + text
    ins = ", ".join(f'"v"({a}), "v"({b})' for a, b in prods)
    if shift_in:
        ins += f', "v"({name_acc}p)'
    acc_c = f'"=&v"({name_acc})' if (first_zero or shift_in) else f'"+v"({name_acc})'
    cnt_c = '"=&v"(cnt)' if counted else '"=&v"(cnt_unused)'
    masks = ", ".join(f'"=&s"(m{q})' for q in range(NM))
    return (f'{indent}asm("{text}"\n{indent}    : {acc_c}, {cnt_c}, {masks}\n'
            f'{indent}    : {ins});\n'), counted


def col_asm_named(n: int, safe: int, first_zero: bool, extras: list[str], shift_in: bool = False):
    """Column text with named operands ([acc], [cnt], [m0..2], [a<p>], [b<p>]) and `extras` -- asm
    lines of the reduction interleaved into the column (fe_mul_red below) -- placed in the wait-state
    slots the column's own schedule would pad with s_nop, else after the column's first
    multiply-add.  Extras never read a mask the column writes, so each one counts as one wait state."""
    sch = schedule(n, safe)
    ex = list(extras)
    # extras beyond the s_nop slots go right after the first multiply-add
    slots = sum(x[1] + 1 for x in sch if x[0] == "nop")
    early, ex = ex[:max(0, len(ex) - slots)], ex[max(0, len(ex) - slots):]
    out = []
    for ins in sch:
        if ins[0] == "nop" and ex:
            k = ins[1] + 1           # wait states this s_nop supplied
            while k > 0 and ex:
                out.append(("x", ex.pop(0)))
                k -= 1
            if k > 0:
                out.append(("nop", k - 1))
            continue
        out.append(ins)
        if ins == ("mad", 0):
            out += [("x", e) for e in early]
    # re-check the mask rule with extras counted as one wait state each
    chk = [("nop", 0) if x[0] == "x" else x for x in out]
    check(chk, n, safe)
    lines, counted = [], 0
    for ins in out:
        if ins[0] == "mad":
            p = ins[1]
            src2 = "0" if (first_zero and p == 0) else "%[acc]"
            lines.append(f"v_mad_u64_u32 %[acc], %[m{p % NM}], %[a{p}], %[b{p}], {src2}")
        elif ins[0] == "cnt":
            m = f"%[m{ins[1] % NM}]"
            prev = "%[cnt]" if counted else "0"
            lines.append(f"v_addc_co_u32 %[cnt], {m}, 0, {prev}, {m}")
            counted += 1
        elif ins[0] == "nop":
            lines.append(f"s_nop {ins[1]}")
        else:
            lines.append(ins[1])
    if shift_in:  # from a separate input: the previous accumulator keeps its low word (a t limb)
        lines.insert(0, "v_lshrrev_b64 %[acc], 32, %[accp]")
    return "\\n\\t".join(lines), counted


# The reduction (kh_math.h fe_reduce512: V_j = h_j*977 + (l_j, l_j+1), W_i = h_i*977 + (h_i-1, h_i),
# R = A + B 2^32) interleaved into fe_mul's last columns: each slice's multiply-add goes into the
# first column statement after its inputs exist, each chain link into the statement after its two
# slices (a 32-bit half of a 64-bit asm operand cannot be named inside the statement that writes
# it).  The links' carry lives in an SGPR pair across statements, so the chain pays no per-link pad.
# (slice name, multiplier t index, addend pair (lo, hi) t indices), in issue order
SLICES = [("V0", 8, (0, 1)), ("W1", 9, (8, 9)), ("V2", 10, (2, 3)), ("W3", 11, (10, 11)),
          ("V4", 12, (4, 5)), ("W5", 13, (12, 13)), ("V6", 14, (6, 7)), ("W7", 15, (14, 15))]
# chain link j: R_j = x + y (+ carry); operands as (slice, half)
LINKS = {1: (("V0", 1), ("W1", 0)), 2: (("V2", 0), ("W1", 1)), 3: (("V2", 1), ("W3", 0)),
         4: (("V4", 0), ("W3", 1)), 5: (("V4", 1), ("W5", 0)), 6: (("V6", 0), ("W5", 1)),
         7: (("V6", 1), ("W7", 0)), 8: (("W7", 1), None)}


def gen_mul_red():
    """fe_mul's columns with the reduction's slices and chain links interleaved (mul_red_cols)."""
    out = ['// R[0..8] = limbs of A + B 2^32 for t = a * b (fe_reduce512\'s slices and chain, interleaved into',
           '// the columns); mk[j] = slice j\'s carry-out mask, r9 = the chain\'s carry out of limb 8',
           '__device__ __forceinline__ void mul_red_cols(const uint32_t *a, const uint32_t *b, uint32_t R[9], uint64_t mk[8],',
           '                                             uint64_t &r9) {',
           '  uint64_t acc, accp, m0, m1, m2, m3, c;',
           '  uint32_t cnt, cnt_unused, t[16];',
           '  uint64_t V0, W1, V2, W3, V4, W5, V6, W7;',
           '  const uint32_t K = 977u;']
    # statement index s: columns 0..14, then F1 (15), F2 (16).  Slice i needs t[mult] and its pair:
    # available after column max(mult, pair hi) -> goes into the next statement.
    ready_slice = {name: max(mu, lo, hi) + 1 for name, mu, (lo, hi) in SLICES}
    # W7 needs t[15] = column 14's high half: statement 15
    ready_slice["W7"] = 15
    place_slice = {}
    for name, _, _ in SLICES:
        place_slice[name] = ready_slice[name]
    # links: after both slices' statements, and after the previous link's statement (carry order)
    place_link = {}
    prev = -1
    for j in range(1, 9):
        x, y = LINKS[j]
        st = max(place_slice[x[0]], place_slice[y[0]] if y else 0) + 1
        st = max(st, prev + 1 if j > 1 else st)
        place_link[j] = st
        prev = st
    nstat = max(place_link.values()) + 1
    sl = {name: (mu, pair) for name, mu, pair in SLICES}
    shift = False
    for st in range(nstat):
        extras, outs, ins = [], [], []
        for name, _, _ in SLICES:
            if place_slice[name] == st:
                mu, (lo, hi) = sl[name]
                j = int(name[1:])
                extras.append(f"v_mad_u64_u32 %[{name}], %[mk{j}], %[t{mu}], %[K], %[p{name}]")
                outs.append(f'[{name}] "=&v"({name}), [mk{j}] "=&s"(mk[{j}])')
                ins.append(f'[t{mu}] "v"(t[{mu}]), [p{name}] "v"(pack64(t[{lo}], t[{hi}]))')
                if '[K] "s"(K)' not in ins:
                    ins.append('[K] "s"(K)')
        for j in range(1, 9):
            if place_link[j] != st:
                continue
            x, y = LINKS[j]
            xs = f"(uint32_t)({x[0]} >> 32)" if x[1] else f"(uint32_t){x[0]}"
            if y:
                ys = f"(uint32_t)({y[0]} >> 32)" if y[1] else f"(uint32_t){y[0]}"
            if j == 1:
                extras.append(f"v_add_co_u32 %[R{j}], %[c], %[x{j}], %[y{j}]")
                outs.append(f'[R{j}] "=&v"(R[{j}]), [c] "=&s"(c)')
            elif j < 8:
                extras.append(f"v_addc_co_u32 %[R{j}], %[c], %[x{j}], %[y{j}], %[c]")
                outs.append(f'[R{j}] "=&v"(R[{j}]), [c] "+s"(c)')
            else:
                extras.append(f"v_addc_co_u32 %[R{j}], %[c], %[x{j}], 0, %[c]")
                outs.append(f'[R{j}] "=&v"(R[{j}]), [c] "+s"(c)')
            ins.append(f'[x{j}] "v"({xs})' + (f', [y{j}] "v"({ys})' if y else ""))
        if st < 15:
            k = st
            prods = [(f"a[{i}]", f"b[{k - i}]") for i in range(8) if 0 <= k - i <= 7]
            safe = len(prods) if k == 0 else (1 if k == 1 else 0)
            # two links in one statement would need a pad between them: never placed so
            text, counted = col_asm_named(len(prods), safe, k == 0, extras, shift_in=shift)
            acc_c = '[acc] "=&v"(acc)' if (k == 0 or shift) else '[acc] "+v"(acc)'
            cnt_c = '[cnt] "=&v"(cnt)' if counted else '[cnt] "=&v"(cnt_unused)'
            o = [acc_c, cnt_c] + [f'[m{q}] "=&s"(m{q})' for q in range(NM)] + outs
            pi = [f'[a{p}] "v"({pa}), [b{p}] "v"({pb})' for p, (pa, pb) in enumerate(prods)] + ins
            if shift:
                out.append("  accp = acc;")
                pi.append('[accp] "v"(accp)')
            out.append(f'  asm("{text}"\n      : {", ".join(o)}\n      : {", ".join(pi)});')
            out.append(f"  t[{k}] = (uint32_t)acc;")
            shift = not counted
            if k < 14:
                if counted:
                    out.append("  acc = (acc >> 32) | ((uint64_t)cnt << 32);")
            else:
                assert counted
                out.append("  t[15] = (uint32_t)(acc >> 32);")
        else:
            # statements after the last column: the remaining slices and links; consecutive links
            # need two wait states between them
            lines = []
            links_here = [e for e in extras if "v_add" in e]
            mads_here = [e for e in extras if "v_mad" in e]
            seq = mads_here[:]
            for i, l in enumerate(links_here):
                if i > 0:
                    seq.append("s_nop 1")
                seq.append(l)
            text = "\\n\\t".join(seq)
            out.append(f'  asm("{text}"\n      : {", ".join(outs)}\n      : {", ".join(ins)});')
    out.append("  R[0] = (uint32_t)V0;")
    out.append("  r9 = c;")
    out.append("  (void)cnt_unused;")
    out.append("}")
    return out


def gen():
    out = ['// kh_cols.h -- GENERATED by tools/gen_cols.py: the product-scanning columns of fe_mul and',
           '// fe_sqr, one asm statement per column, scheduled so that every carry count reads a mask',
           '// written >= 2 instructions earlier (no s_nop inside a column).  See the generator.',
           '// Included by kh_math.h inside namespace kh (device compilation only).',
           '#pragma once', '', '#if defined(__HIP_DEVICE_COMPILE__)', '']
    # fe_mul: t = a * b (16 limbs)
    out.append('// t[0..15] = a * b')
    out.append('__device__ __forceinline__ void mul_cols(const uint32_t *a, const uint32_t *b, uint32_t t[16]) {')
    out.append('  uint64_t acc, accp, m0, m1, m2, m3;')
    out.append('  uint32_t cnt, cnt_unused;')
    shift = False
    for k in range(15):
        prods = [(f"a[{i}]", f"b[{k - i}]") for i in range(8) if 0 <= k - i <= 7]
        # column 0 and the first product of column 1 cannot carry: (2^32-1)^2 + 2^32 - 1 < 2^64
        safe = len(prods) if k == 0 else (1 if k == 1 else 0)
        if shift:
            out.append("  accp = acc;")
        s, counted = emit_column("acc", prods, safe, k == 0, shift_in=shift)
        out.append(s.rstrip("\n"))
        out.append(f"  t[{k}] = (uint32_t)acc;")
        shift = not counted
        if counted:
            out.append("  acc = (acc >> 32) | ((uint64_t)cnt << 32);")
    out.append("  t[15] = (uint32_t)acc;")
    out.append("  (void)cnt_unused;")
    out.append("}")
    out.append("")
    # fe_sqr cross products a_i * a_j, i < j: columns 1..13 (t[0] = 0, t[14..15] from the last acc)
    out.append('// t[1..15] = sum_{i<j} a_i a_j 2^(32(i+j)) (t[0] = 0): the cross products of a square, not doubled')
    out.append('__device__ __forceinline__ void sqr_cross_cols(const uint32_t *a, uint32_t t[16]) {')
    out.append('  uint64_t acc, accp, m0, m1, m2, m3;')
    out.append('  uint32_t cnt, cnt_unused;')
    out.append('  t[0] = 0;')
    shift = False
    for k in range(1, 14):
        prods = [(f"a[{i}]", f"a[{k - i}]") for i in range(8) if i < k - i <= 7]
        # columns 1 and 2 hold one cross product each and column 3 starts on an accumulator of at
        # most 2^32 - 1: their first products cannot carry
        safe = 1 if k <= 3 else 0
        if shift:
            out.append("  accp = acc;")
        s, counted = emit_column("acc", prods, safe, k == 1, shift_in=shift)
        out.append(s.rstrip("\n"))
        out.append(f"  t[{k}] = (uint32_t)acc;")
        shift = not counted
        if counted:
            out.append("  acc = (acc >> 32) | ((uint64_t)cnt << 32);")
    assert not shift
    out.append("  t[14] = (uint32_t)acc;")
    out.append("  t[15] = (uint32_t)(acc >> 32);")
    out.append("  (void)cnt_unused;")
    out.append("}")
    out.append("")
    out += gen_mul_red()
    out += ["#endif"]
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(gen(), end="")
