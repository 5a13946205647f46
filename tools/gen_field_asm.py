#!/usr/bin/env python3
"""Generate tools/kh_field_asm.h: secp256k1 field multiplication and squaring for gfx950 as single
inline-asm statements (development study; the engine keeps hipcc's code).

Why: gfx950 needs 2 wait states between a VALU instruction that writes an SGPR carry mask and a
VALU instruction that reads it (v_add_co -> v_addc).  hipcc pads every such pair in a carry chain
with s_nop, and pads every inline-asm boundary, so the C/asm-per-product form of fe_mul issued about
two s_nop per partial product.  Here the whole product + reduction is one statement whose carry
reads are scheduled >= 2 instructions after their writes (three rotating SGPR pairs), and a paired
form interleaves two independent multiplications instruction by instruction.

Arithmetic (same value as kh_math.h's portable fe_mul / fe_sqr, secp256k1/IntMod.cpp:855-1093):
  product: 8x32-bit limbs, product scanning; column sums in a 64-bit VGPR pair, their carries
           counted in a third register (v_addc_co_u32 from the v_mad_u64_u32 carry-out);
  squaring: cross products by product scanning, doubled with v_alignbit, squares added per limb;
  fold 1: u = t_lo + t_hi*977 + t_hi<<32   (2^256 == 2^32 + 977 mod p), 64-bit accumulator,
          additions of 32-bit words as v_mad_u64_u32 by 1 (no carry flags);
  fold 2: r = u_lo + h*977 + h<<32 with h = u >> 256 (< 2^34), limbs 0..2 exactly, limb 3 gets the
          carry with a wrapping add.
  The statement returns a flag word = max(and(r2..r7), u3): it is 0xFFFFFFFF only if limb 3 could
  have carried on (u3 = ~0) or the result may be >= p (r2..r7 all ones); the caller then recomputes
  with the portable code (probability ~2^-32 per product).
The two 64-bit accumulator pairs per product are fixed VGPRs named in the clobber list, so pairs and
their halves can both be addressed in the text; everything else is compiler-allocated operands.
Result on the MI355X: 16% fewer cycles per multiplication in isolation (tools/ubench_field4.hip),
no gain inside the BSGS walk (opaque to hipcc's scheduler; the paired form spills).
"""
import os
import sys

P_977 = "%[k977]"  # VOP3 takes no literal on gfx9: 977 comes in an SGPR operand


class Stream:
    """One multiplication/squaring: an instruction list over named registers."""

    def __init__(self, tag, vbase):
        self.tag = tag
        self.ins = []          # (text, sgpr_writes, sgpr_reads)
        self.vbase = vbase     # first fixed scratch VGPR: T[0..15] = vbase..vbase+15, A, B pairs after
        # the 512-bit intermediate lives in compiler-allocated operands; only the two accumulator
        # pairs are fixed registers (their halves must be addressable)
        self.T = [f"%[{tag}t{i}]" for i in range(16)]
        self.A = (f"v{vbase}", f"v{vbase + 1}")
        self.B = (f"v{vbase + 2}", f"v{vbase + 3}")
        self.c = [f"%[{tag}c{i}]" for i in range(3)]
        self.cn = 0

    @staticmethod
    def pair(p):
        lo = int(p[0][1:])
        return f"v[{lo}:{lo + 1}]"

    def emit(self, text, w=(), r=()):
        self.ins.append((text, tuple(w), tuple(r)))

    def next_c(self):
        c = self.c[self.cn % 3]
        self.cn += 1
        return c

    # ---------------------------------------------------------------- product scanning
    def column(self, prods, X, cnt, fresh_cnt, extra_after_last=()):
        """X (pair) += sum a*b over prods; carries counted into register cnt (zeroed first if
        fresh_cnt).  extra_after_last: carry-independent instructions placed after the last mad."""
        pend = []  # carry sgpr of mads whose addc is pending
        first_cnt = fresh_cnt
        n = len(prods)

        def do_addc():
            nonlocal first_cnt
            c = pend.pop(0)
            if first_cnt:
                self.emit(f"v_cndmask_b32_e64 {cnt}, 0, 1, {c}", r=(c,))
                first_cnt = False
            else:
                self.emit(f"v_addc_co_u32_e64 {cnt}, {c}, 0, {cnt}, {c}", w=(c,), r=(c,))

        for k, (x, y) in enumerate(prods):
            c = self.next_c()
            self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c}, {x}, {y}, {self.pair(X)}", w=(c,))
            pend.append(c)
            if k == n - 1:
                for e in extra_after_last:
                    self.emit(e)
            if len(pend) >= 3 or (k == n - 1):
                pass
            while len(pend) >= 3:
                do_addc()
        while pend:
            do_addc()

    def product(self, a, b):
        """t = a*b (512 bits) into T[0..15]."""
        T, A, B = self.T, self.A, self.B
        # column 0: one product, no carry possible
        self.emit(f"v_mad_u64_u32 {self.pair(A)}, {self.next_c()}, {a[0]}, {b[0]}, 0", w=(self.c[0],))
        # A = (t0, hi0); next column accumulates in B = (hi0, cnt)
        self.emit(f"v_mov_b32 {T[0]}, {A[0]}")
        self.emit(f"v_mov_b32 {B[0]}, {A[1]}")
        self.emit(f"v_mov_b32 {B[1]}, 0")
        X, Y = B, A
        for k in range(1, 15):
            prods = [(a[i], b[k - i]) for i in range(8) if 0 <= k - i <= 7]
            if k == 14:
                # last column: no carry out of 2^512
                for (x, y) in prods:
                    self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {x}, {y}, {self.pair(X)}")
                self.emit(f"v_mov_b32 {T[14]}, {X[0]}")
                self.emit(f"v_mov_b32 {T[15]}, {X[1]}")
                break
            # carries of this column go to Y.hi; afterwards Y = (X.hi, cnt) and t_k = X.lo
            self.column(prods, X, Y[1], True,
                        extra_after_last=(f"v_mov_b32 {T[k]}, {X[0]}", f"v_mov_b32 {Y[0]}, {X[1]}"))
            X, Y = Y, X
        self._fix_sgpr_writes()

    def square(self, a):
        """t = a^2 (512 bits) into T[0..15]."""
        T, A, B = self.T, self.A, self.B
        # cross products sum_{i<j} a_i a_j 2^(32(i+j)) into T[1..14]
        self.emit(f"v_mad_u64_u32 {self.pair(A)}, {self.next_c()}, {a[0]}, {a[1]}, 0")
        self.emit(f"v_mov_b32 {T[1]}, {A[0]}")
        self.emit(f"v_mov_b32 {B[0]}, {A[1]}")
        self.emit(f"v_mov_b32 {B[1]}, 0")
        X, Y = B, A
        for k in range(2, 14):
            prods = [(a[i], a[k - i]) for i in range(8) if i < k - i <= 7]
            if k == 13:
                for (x, y) in prods:
                    self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {x}, {y}, {self.pair(X)}")
                self.emit(f"v_mov_b32 {T[13]}, {X[0]}")
                self.emit(f"v_mov_b32 {T[14]}, {X[1]}")
                break
            self.column(prods, X, Y[1], True,
                        extra_after_last=(f"v_mov_b32 {T[k]}, {X[0]}", f"v_mov_b32 {Y[0]}, {X[1]}"))
            X, Y = Y, X
        # double: T = 2 * cross (T0 = 0, T15 = T14 >> 31)
        self.emit(f"v_lshrrev_b32 {T[15]}, 31, {T[14]}")
        for i in range(14, 1, -1):
            self.emit(f"v_alignbit_b32 {T[i]}, {T[i]}, {T[i - 1]}, 31")
        self.emit(f"v_lshlrev_b32 {T[1]}, 1, {T[1]}")
        # add the squares limb by limb through a 64-bit accumulator X (sum stays < 2^64):
        # limb 2i: X += a_i^2 + T[2i]; limb 2i+1: X += T[2i+1]
        X = A
        for i in range(8):
            if i == 0:
                self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {a[0]}, {a[0]}, 0")
                # T0 = 0: limb 0 is X.lo
            else:
                self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {a[i]}, {a[i]}, {self.pair(X)}")
                self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {T[2 * i]}, 1, {self.pair(X)}")
            self.emit(f"v_mov_b32 {T[2 * i]}, {X[0]}")
            self.emit(f"v_lshrrev_b64 {self.pair(X)}, 32, {self.pair(X)}")
            self.emit(f"v_mad_u64_u32 {self.pair(X)}, {self.next_c()}, {T[2 * i + 1]}, 1, {self.pair(X)}")
            self.emit(f"v_mov_b32 {T[2 * i + 1]}, {X[0]}")
            if i < 7:
                self.emit(f"v_lshrrev_b64 {self.pair(X)}, 32, {self.pair(X)}")
        self._fix_sgpr_writes()

    def _fix_sgpr_writes(self):
        # every v_mad_u64_u32 writes its carry operand: record it for the hazard pass
        out = []
        for (t, w, r) in self.ins:
            if t.startswith("v_mad_u64_u32") and not w:
                w = (t.split(",")[1].strip(),)
            out.append((t, w, r))
        self.ins = out

    def reduce(self, r_ops, flag_op):
        """T (512 bits) -> r (8 operands), flag (see module docstring)."""
        T, X, Y = self.T, self.A, self.B
        c = lambda: self.next_c()
        # fold 1 into T[0..7] (u_i), h in X
        self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[8]}, {P_977}, 0")
        self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[0]}, 1, {self.pair(X)}")
        self.emit(f"v_mov_b32 {T[0]}, {X[0]}")
        self.emit(f"v_lshrrev_b64 {self.pair(X)}, 32, {self.pair(X)}")
        for i in range(1, 8):
            self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[8 + i]}, {P_977}, {self.pair(X)}")
            self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[i]}, 1, {self.pair(X)}")
            self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[7 + i]}, 1, {self.pair(X)}")
            self.emit(f"v_mov_b32 {T[i]}, {X[0]}")
            self.emit(f"v_lshrrev_b64 {self.pair(X)}, 32, {self.pair(X)}")
        self.emit(f"v_mad_u64_u32 {self.pair(X)}, {c()}, {T[15]}, 1, {self.pair(X)}")
        # fold 2: h = X (< 2^35)
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {X[0]}, {P_977}, 0")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {T[0]}, 1, {self.pair(Y)}")
        self.emit(f"v_mov_b32 {r_ops[0]}, {Y[0]}")
        self.emit(f"v_lshrrev_b64 {self.pair(Y)}, 32, {self.pair(Y)}")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {T[1]}, 1, {self.pair(Y)}")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {X[0]}, 1, {self.pair(Y)}")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {X[1]}, {P_977}, {self.pair(Y)}")
        self.emit(f"v_mov_b32 {r_ops[1]}, {Y[0]}")
        self.emit(f"v_lshrrev_b64 {self.pair(Y)}, 32, {self.pair(Y)}")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {T[2]}, 1, {self.pair(Y)}")
        self.emit(f"v_mad_u64_u32 {self.pair(Y)}, {c()}, {X[1]}, 1, {self.pair(Y)}")
        self.emit(f"v_mov_b32 {r_ops[2]}, {Y[0]}")
        self.emit(f"v_lshrrev_b64 {self.pair(Y)}, 32, {self.pair(Y)}")
        self.emit(f"v_add_u32 {r_ops[3]}, {T[3]}, {Y[0]}")
        for i in range(4, 8):
            self.emit(f"v_mov_b32 {r_ops[i]}, {T[i]}")
        self.emit(f"v_and_b32 {flag_op}, {r_ops[2]}, {r_ops[3]}")
        self.emit(f"v_bitop3_b32 {flag_op}, {flag_op}, {r_ops[4]}, {r_ops[5]} bitop3:0x80")
        self.emit(f"v_bitop3_b32 {flag_op}, {flag_op}, {r_ops[6]}, {r_ops[7]} bitop3:0x80")
        self.emit(f"v_max_u32 {flag_op}, {flag_op}, {T[3]}")
        self._fix_sgpr_writes()


def schedule(streams):
    """Interleave the streams round-robin and pad SGPR write->read distances to >= 2."""
    seq = []
    idx = [0] * len(streams)
    while any(idx[s] < len(st.ins) for s, st in enumerate(streams)):
        for s, st in enumerate(streams):
            if idx[s] < len(st.ins):
                seq.append(st.ins[idx[s]])
                idx[s] += 1
    out = []
    last_write = {}
    pos = 0
    for (t, w, r) in seq:
        for reg in r:
            if reg in last_write:
                gap = pos - last_write[reg] - 1
                if gap < 2:
                    out.append(f"s_nop {1 - gap}")
                    pos += 2 - gap
        out.append(t)
        for reg in w:
            last_write[reg] = pos
        pos += 1
    return out


def fe_ops(name):
    return [f"%[{name}{i}]" for i in range(8)]


def gen_function(fname, kind, nstreams, part="all"):
    """kind: 'mul' or 'sqr'.  part (timing experiments only): 'all', 'prod' (no reduction: r = t_lo),
    'red' (reduction of t = a || b)."""
    vbases = [124, 120][:nstreams]
    streams = []
    for s in range(nstreams):
        st = Stream(f"s{s}", vbases[s])
        a = fe_ops(f"a{s}_")
        b = fe_ops(f"b{s}_")
        if part == "red":
            for i in range(8):
                st.emit(f"v_mov_b32 {st.T[i]}, {a[i]}")
                st.emit(f"v_mov_b32 {st.T[8 + i]}, {b[i]}")
        elif kind == "mul":
            st.product(a, b)
        else:
            st.square(a)
        if part == "prod":
            r = fe_ops(f"r{s}_")
            for i in range(8):
                st.emit(f"v_add_u32 {r[i]}, {st.T[i]}, {st.T[8 + i]}")
            st.emit(f"v_mov_b32 %[f{s}], 0")
        else:
            st.reduce(fe_ops(f"r{s}_"), f"%[f{s}]")
        streams.append(st)
    body = schedule(streams)
    clob = []
    for vb in vbases:
        clob += [f'"v{vb + i}"' for i in range(4)]
    outs, ins = [], ['[k977] "s"(977u)']
    for s in range(nstreams):
        outs += [f'[r{s}_{i}] "=&v"(r{s}.d[{i}])' for i in range(8)]
        outs.append(f'[f{s}] "=&v"(f{s})')
        outs += [f'[s{s}c{i}] "=&s"(c{s}_{i})' for i in range(3)]
        outs += [f'[s{s}t{i}] "=&v"(t{s}[{i}])' for i in range(16)]
        ins += [f'[a{s}_{i}] "v"(a{s}.d[{i}])' for i in range(8)]
        if kind == "mul":
            ins += [f'[b{s}_{i}] "v"(b{s}.d[{i}])' for i in range(8)]
    args = []
    for s in range(nstreams):
        args.append(f"fe &r{s}")
        args.append(f"const fe &a{s}")
        if kind == "mul":
            args.append(f"const fe &b{s}")
    lines = []
    n_instr = sum(1 for x in body if not x.startswith("s_nop"))
    n_nop = sum(1 for x in body if x.startswith("s_nop"))
    lines.append(f"// {kind} x{nstreams}: {n_instr} instructions, {n_nop} s_nop")
    lines.append(f"__device__ __forceinline__ uint32_t {fname}({', '.join(args)}) {{")
    fl = ", ".join(f"f{s}" for s in range(nstreams))
    lines.append(f"  uint32_t {fl};")
    lines.append("#if defined(__HIP_DEVICE_COMPILE__)")
    for s in range(nstreams):
        lines.append(f"  uint64_t c{s}_0, c{s}_1, c{s}_2;")
        lines.append(f"  uint32_t t{s}[16];")
    lines.append("  asm volatile(")
    for t in body:
        lines.append(f'      "{t}\\n"')
    lines.append(f"      : {', '.join(outs)}")
    lines.append(f"      : {', '.join(ins)}")
    lines.append(f"      : {', '.join(clob)});")
    lines.append("#else")
    lines.append("  " + " ".join(f"f{s} = 0xFFFFFFFFu;" for s in range(nstreams)) + "  // host pass: never called")
    lines.append("  " + " ".join(f"(void)r{s}; (void)a{s};" + (f" (void)b{s};" if kind == "mul" else "") for s in range(nstreams)))
    lines.append("#endif")
    if nstreams == 1:
        lines.append("  return f0;")
    else:
        lines.append("  return f0 > f1 ? f0 : f1;")
    lines.append("}")
    return "\n".join(lines)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "kh_field_asm.h")
    parts = ["// GENERATED by tools/gen_field_asm.py -- do not edit.  See that file for the algorithm.",
             "// Device-only: secp256k1 field mul/sqr as single gfx950 inline-asm statements.",
             "#pragma once", "#if defined(__HIPCC__)", "namespace kh {"]
    parts.append(gen_function("fe_mul_asm", "mul", 1))
    parts.append(gen_function("fe_mul2_asm", "mul", 2))
    parts.append(gen_function("fe_sqr_asm", "sqr", 1))
    parts.append(gen_function("fe_sqr2_asm", "sqr", 2))
    if os.environ.get("KH_GEN_EXPERIMENTS"):
        parts.append(gen_function("fe_mulP_asm", "mul", 1, "prod"))
        parts.append(gen_function("fe_red_asm", "mul", 1, "red"))
    parts += ["}  // namespace kh", "#endif"]
    open(out, "w").write("\n\n".join(parts) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
