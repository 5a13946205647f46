#!/usr/bin/env python3
"""Class-weighted VALU ceiling of the walk kernels (bench.py "frac_mix").

For each kernel: the dynamic instruction mix per point, priced at the measured SIMD cost of each
instruction class, gives the SIMD cycles per point the kernel needs when every SIMD issues its mix
back to back (s_nop pads included); bench.py compares the measured rate with
1024 SIMDs x clock / that figure.

Dynamic mix.  The hot loops are read from the ISA listing of an analysis build compiled with
-DKH_ISA_MARKS, which only adds an empty asm comment ";@kh_rare" to every rarely executed fix-up
block (kh_math.h KH_RARE_MARK: carries rippling past limb 1, reductions with an overflowing slice,
recorded hits).  A rare region runs from a marked block to the label its guarding branch jumps to;
everything else in the loop is the common path, executed once per trip.  Per point:
    (forward-loop trip + backward-loop trip) / 2
since both loops of a 2H-point group run H trips (one prefix product / one symmetric pair each); the
hash walks' per-point side loop inside the backward loop counts once per point;
the inversion and the centre step (once per group) are left out (< 1 %: they are checked against the
PMC count below).  The sparse BSGS pad rebuilds every other prefix product in the backward loop
(SPARSE, kh_kernels.hip), a block taken on half the trips: the tool counts it at 1/2 when it finds
it (a branch on the loop counter's parity, s_bitcmp).  The resulting VALU per point is printed beside
the PMC SQ_INSTS_VALU per point of the shipped build; they agree within a few %.

Class costs (SIMD cycles per wave-instruction at 4 waves/SIMD, in shader cycles, whole-launch
throughput): profiles/r03e_ubench_cost.txt (tools/ubench_cost.hip).  On gfx950 they fall in two
rates: ~2.2 cycles (32-bit add / logic / shifts / v_mov_b32 / v_bitop3: a wave64 over a SIMD-32) and
~4.2 (v_mad_u64_u32, every carry-in/out op, v_alignbit, v_add3, v_perm, packed 16-bit ops, compares,
v_cndmask, 64-bit ALU ops, 32-bit multiplies); an s_nop stream issues at ~1.1 cycles per wait state.

Floor (round 4; what bench.py's frac_mix divides by, so that it is a bound): every class at the
hardware's own issue floor instead of its measured single-class cost -- 2 cycles for a full-rate
wave64 instruction (MI355X_MICROARCH.md: 32 lanes per cycle), 4 for a half-rate one -- an s_nop wait
state at its in-situ cost (ubench "mad,nop,addc,nop" against "mad+addc, hazards scheduled": the
cycles the pads add when other waves issue beside them, ~0.3), and the share of VALU instructions
the PMC saw dual-issued (SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU) taken as free.  A kernel cannot issue
its instructions faster than that at a given clock, whatever their order.

Quad model (round 4, what the walks actually meet): on gfx950 a full-rate instruction only issues in
2 cycles when another full-rate one shares its 4-cycle quad; streams that mix full- and half-rate
instructions -- alternating, or in runs of 2, 4 or 16 -- issue at ~4 cycles per instruction whatever
their classes (profiles/r04d_ubench_cost.txt "alignbit + v_add_u32 mix" 4.04, "alignbit + bitop3 mix"
3.86, r04e_ubench_runs.txt "runs" 4.00-4.04 at 4 waves/SIMD).  simd_cycles_per_point_quad prices
every VALU instruction at one quad, the dual-issued share (SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU) free
and s_nop at its in-situ cost.  It is a model of the mixed kernels, not a hardware bound: pure
full-rate stretches issued by several waves at once would beat it.

usage: python tools/valu_mix.py LISTING.s PMC_SUMMARY.json OUT.json [COST.txt]
"""
import json
import re
import sys

# kernel -> (symbol, its largest loop runs once per point: the hash walks' side loop, prefix
# products per forward-loop trip: the deferred-probe walks pair two per trip, kh_kernels.hip)
# (symbol, per-point side loop, prefix products per forward trip, backward steps per trip: the
# sparse-pad walks run two steps, odd then even, per backward trip since round 4's kept row)
KERNELS = {"k_walk<7, 2048>": ("_Z6k_walkILi7ELi2048EEv9walk_args", False, 2, 2),
           "k_walk<10, 2048>": ("_Z6k_walkILi10ELi2048EEv9walk_args", False, 2, 2),
           "k_walk<11, 2048>": ("_Z6k_walkILi11ELi2048EEv9walk_args", True, 1, 1)}

# ubench_cost.txt pattern name -> class
PATTERN = {"mad_u64_u32 acc, 4 chains": "mad64", "add_co/addc, 4 sgpr chains": "carry", "v_mov_b32": "mov",
           "v_add_u32": "full", "v_bitop3_b32": "bitop3", "v_alignbit_b32": "alignbit", "v_add3_u32": "add3",
           "v_pk_lshlrev_b16": "pk16", "v_perm_b32": "perm", "v_cmp_eq_u32 (vcc)": "cmp",
           "v_cndmask_b32_e64 (sgpr)": "cndmask", "v_add_co_u32_e32 (vcc) indep": "carry_vcc",
           "v_lshrrev_b64": "alu64", "v_mov_b64": "mov64", "v_mul_lo/hi_u32": "mul32", "s_nop 0 only": "s_nop"}


def klass(op: str) -> str | None:
    """Cost class of one opcode (None: not a VALU / s_nop instruction)."""
    if op == "s_nop":
        return "s_nop"
    if not op.startswith("v_"):
        return None
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith(("v_add_co_u32", "v_sub_co_u32", "v_subrev_co_u32")):
        return "carry_vcc" if op.endswith("_e32") else "carry"
    if op.startswith(("v_addc_co_u32", "v_subb_co_u32", "v_subbrev_co_u32")):
        return "carry_vcc" if op.endswith("_e32") else "carry"
    if op.startswith(("v_mov_b64", "v_pk_mov_b32")):
        return "mov64"
    if op.startswith("v_mov_b32"):
        return "mov"
    if op.startswith("v_bitop3"):
        return "bitop3"
    if op.startswith(("v_alignbit", "v_alignbyte")):
        return "alignbit"
    if op.startswith(("v_add3_u32", "v_lshl_add_u32", "v_add_lshl_u32", "v_lshl_or_b32", "v_and_or_b32",
                      "v_or3_b32", "v_xor3_b32", "v_xad_u32", "v_bfi_b32", "v_bfe_u32")):
        return "add3"
    if op.startswith("v_pk_"):
        return "pk16"
    if op.startswith("v_perm"):
        return "perm"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "cmp"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_lshrrev_b64", "v_lshlrev_b64", "v_ashrrev_i64", "v_lshl_add_u64")):
        return "alu64"
    if op.startswith(("v_mul_lo", "v_mul_hi", "v_mad_u32", "v_mul_u32")):
        return "mul32"
    if op.startswith(("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32",
                      "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_max_u32", "v_min_u32")):
        return "full"
    return "other"  # priced as the half-rate median


def costs(path: str) -> dict:
    """{class: SIMD cycles per wave-instruction at 4 waves/SIMD} from ubench_cost.txt: the "span"
    figure (whole launch, in-kernel clock), i.e. the SIMD's throughput for that class."""
    c = {}
    for line in open(path):
        m = re.match(r"^(.*?)\s+W1 span\s+([\d.]+).*W4 span\s+([\d.]+)", line)
        if m and m.group(1).strip() in PATTERN:
            c[PATTERN[m.group(1).strip()]] = float(m.group(3))
    half = sorted(v for k, v in c.items() if k in ("mad64", "carry", "cmp", "alignbit", "add3", "perm", "alu64"))
    c["other"] = half[len(half) // 2]
    return c


FULL_RATE = ("mov", "full", "bitop3")  # 2-cycle wave64 issue; every other VALU class is half rate


def nop_in_situ(path: str) -> float:
    """SIMD cycles an s_nop wait state adds between half-rate instructions at 4 waves/SIMD: 16 of the
    32 instructions of "mad,nop,addc,nop" are pads, "mad+addc, hazards scheduled" has none."""
    span = {}
    for line in open(path):
        m = re.match(r"^(.*?)\s+W1 span\s+([\d.]+).*W4 span\s+([\d.]+)", line)
        if m:
            span[m.group(1).strip()] = float(m.group(3))
    padded, plain = span["mad,nop,addc,nop (as hipcc)"], span["mad+addc, hazards scheduled"]
    return max(0.0, (32 * padded - 16 * plain) / 16)


def floor_costs(classes, nop: float) -> dict:
    return {k: (nop if k == "s_nop" else 2.0 if k in FULL_RATE else 4.0) for k in classes}


def function(lines, sym):
    s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[s:e]


def blocks(body):
    """[(label, [instruction lines], marked)] in listing order; label None for fall-through blocks."""
    out, cur, lab, mark = [], [], None, False
    for l in body:
        t = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m or t.startswith("; %bb."):
            if cur or lab:
                out.append((lab, cur, mark))
            cur, lab, mark = [], (m.group(1) if m else None), False
            continue
        if ";@kh_rare" in t:
            mark = True
            continue
        if t and not t.startswith(";") and not t.startswith(".") and not t.endswith(":"):
            cur.append(t)
    out.append((lab, cur, mark))
    return out


def loops(bl):
    """(start, end) block indices of each loop (a backward branch to a label), largest first."""
    idx = {b[0]: i for i, b in enumerate(bl) if b[0]}
    res = []
    for i, (_, ins, _) in enumerate(bl):
        for t in ins:
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", t)
            if m and m.group(2) in idx and idx[m.group(2)] <= i:
                res.append((idx[m.group(2)], i))
    # keep outermost-distinct loops by size
    res = sorted(set(res), key=lambda x: -(sum(len(bl[k][1]) for k in range(x[0], x[1] + 1))))
    return res


def common_path(bl, a, b):
    """Per-trip weight of each block of the loop [a, b]: 0 for rare regions, 1/2 for the parity
    block, else 1."""
    w = [1.0] * len(bl)
    idx = {x[0]: i for i, x in enumerate(bl) if x[0]}
    # the sparse pad's odd-trip block: entered through a branch on the counter's parity (s_bitcmp)
    for j in range(a, b + 1):
        ins = bl[j][1]
        if ins and any(t.startswith("s_bitcmp") for t in ins):
            m = re.match(r"s_cbranch_scc[01]\s+(\.LBB\d+_\d+)", ins[-1])
            if m and idx.get(m.group(1), -1) > j:
                for k in range(j + 1, min(idx[m.group(1)], b + 1)):
                    w[k] = 0.5
    # rare regions: the blocks of [a, b] that the loop reaches only through a marked block.  A walk
    # of the control-flow graph from the loop's first block that never enters a marked block (the
    # compiler may lay a rare block out before its join, so layout order alone does not bound it)
    def succ(k):
        ins = bl[k][1]
        out = []
        last = ins[-1] if ins else ""
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", last)
        if m and m.group(2) in idx:
            out.append(idx[m.group(2)])
        if not last.startswith("s_branch") and k + 1 <= b:
            out.append(k + 1)
        return out
    seen, todo = {a}, [a]
    while todo:
        k = todo.pop()
        for s in succ(k):
            if a <= s <= b and s not in seen and not bl[s][2]:
                seen.add(s)
                todo.append(s)
    for k in range(a, b + 1):
        if k not in seen:
            w[k] = 0.0
    return w


def mix(listing: str, sym: str, per_point_loop: bool, fwd_per_trip: int = 1, bwd_per_trip: int = 1):
    """Lane-instructions per point by class.  The largest loop of the kernel is its per-pair
    backward loop (deferred-probe walks) or, with per_point_loop, the per-point side loop of the
    hash walks inside it; loops overlapping it are the rest of the backward loop (per pair), and the
    largest loop before it is the forward loop (per prefix product = per pair)."""
    lines = open(listing).read().split("\n")
    bl = blocks(function(lines, sym))
    ls = loops(bl)
    top = ls[0]
    over = [x for x in ls if not (x[1] < top[0] or x[0] > top[1])]
    lo, hi = min(x[0] for x in over), max(x[1] for x in over)
    fwd = next(x for x in ls if x[1] < lo)
    weight = {}
    for k in range(fwd[0], fwd[1] + 1):
        weight[k] = 0.5 / fwd_per_trip  # a trip makes fwd_per_trip prefix products (2 points each)
    for k in range(lo, hi + 1):
        weight[k] = 1.0 if (per_point_loop and top[0] <= k <= top[1]) else 0.5 / bwd_per_trip
    # one control-flow walk over the whole backward loop (its nested ranges share the header lo)
    cp = [common_path(bl, lo, hi), common_path(bl, fwd[0], fwd[1])]
    rare = {k for w in cp for k in range(len(w)) if w[k] == 0.0}
    half = {k for w in cp for k in range(len(w)) if w[k] == 0.5}
    per_point = {}
    for k, wt in weight.items():
        if k in rare:
            continue
        if k in half:
            wt *= 0.5
        for t in bl[k][1]:
            op = t.split()[0]
            c = klass(op)
            if c is None:
                continue
            n = wt
            if c == "s_nop":
                n *= int(t.split()[1]) + 1 if len(t.split()) > 1 else 1  # s_nop N = N + 1 states
            per_point[c] = per_point.get(c, 0.0) + n
    return per_point


def main():
    listing, pmc, out = sys.argv[1:4]
    cost_path = sys.argv[4] if len(sys.argv) > 4 else "profiles/r03e_ubench_cost.txt"
    cost = costs(cost_path)
    nop = nop_in_situ(cost_path)
    pm = json.load(open(pmc))
    res = {}
    for name, (sym, ppl, fpt, bpt) in KERNELS.items():
        pp = mix(listing, sym, ppl, fpt, bpt)
        # pp: lane-instructions per point (every lane walks its own points); a wave-instruction
        # serves 64 points, so SIMD cycles per point = sum(count x class cost) / 64
        valu = sum(v for k, v in pp.items() if k != "s_nop")
        cyc = sum(v * cost[k] for k, v in pp.items()) / 64
        e = {"valu_per_point_static": valu, "s_nop_states_per_point": pp.get("s_nop", 0.0),
             "lane_instructions_per_point": {k: round(v, 2) for k, v in sorted(pp.items())},
             "class_cost_simd_cycles": {k: cost[k] for k in sorted(pp)},
             "simd_cycles_per_point": cyc,
             "simd_cycles_by_class": {k: round(v * cost[k] / 64, 4)
                                      for k, v in sorted(pp.items(), key=lambda x: -x[1] * cost[x[0]])},
             "listing": listing, "costs": cost_path,
             "recompute": "simd_cycles_per_point = sum(lane_instructions_per_point[c] * class_cost_simd_cycles[c]) / 64 * pmc_over_static"}
        fl = floor_costs(pp, nop)
        cyc_floor = sum(v * fl[k] for k, v in pp.items()) / 64
        e.update(class_floor_simd_cycles=fl, s_nop_in_situ_cycles=nop)
        dual = 0.0
        f = 1.0
        if name in pm and "valu_lane_instructions_per_point" in pm[name]:
            e["valu_per_point_pmc"] = pm[name]["valu_lane_instructions_per_point"]
            # scale the static mix to the measured dynamic VALU count (inversion, centre step)
            f = pm[name]["valu_lane_instructions_per_point"] / valu
            e["pmc_over_static"] = f
            e["simd_cycles_per_point"] = cyc * f
            c = pm[name].get("counters_per_dispatch", {})
            if c.get("SQ_ACTIVE_INST_VALU2") and c.get("SQ_INSTS_VALU"):
                dual = c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"]
        e["dual_issue_share"] = dual
        e["simd_cycles_per_point_floor"] = cyc_floor * f * (1 - dual)
        e["simd_cycles_per_point_quad"] = (valu * f * 4.0 * (1 - dual) + pp.get("s_nop", 0.0) * nop) / 64
        e["recompute_quad"] = ("simd_cycles_per_point_quad = (valu_per_point_pmc * 4 * (1 - dual_issue_share) + "
                               "s_nop_states_per_point * s_nop_in_situ_cycles) / 64")
        e["recompute_floor"] = ("simd_cycles_per_point_floor = sum(lane_instructions_per_point[c] * "
                                "class_floor_simd_cycles[c]) / 64 * pmc_over_static * (1 - dual_issue_share)")
        res[name] = e
    json.dump(res, open(out, "w"), indent=1)
    for k, e in res.items():
        print(k, "static VALU/pt %.1f  PMC %.1f  s_nop states/pt %.1f  SIMD cycles/pt %.3f (floor %.3f, quad %.3f)" % (
            e["valu_per_point_static"], e.get("valu_per_point_pmc", 0), e["s_nop_states_per_point"],
            e["simd_cycles_per_point"], e["simd_cycles_per_point_floor"], e["simd_cycles_per_point_quad"]))
        print("   ", e["simd_cycles_by_class"])


if __name__ == "__main__":
    main()
