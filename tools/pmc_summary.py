"""Aggregate rocprofv3 --pmc passes (<src>/<pass>/run_counter_collection.csv) into a per-kernel summary:
counters per dispatch and per point, HBM bytes with the MI355X_MICROARCH.md corrections, and the
VALU issue rate.

HBM (guide, HBM section): reads = TCC_EA0_RDREQ x 64 B, writes = WRITE_SIZE x 1 KiB (exact for 16-B
per-lane streaming stores).  On gfx950 a wide coalesced read (16 B/lane, the inversion pad's
loads) is tallied at HALF its bytes, so the pad's read bytes are counted separately: the pad is
written once and read back once per group, so its read bytes equal the dispatch's write bytes
(WRITE_SIZE; the few hit/candidate records are noise).  Then
  pad_read      = WRITE_SIZE x 1 KiB                    (exact)
  other_read    = TCC_EA0_RDREQ x 64 B - pad_read / 2    (the probes' random 16-B loads: 64 B each)
  hbm_bytes     = other_read + pad_read + pad_write.
VALU: SQ_INSTS_VALU counts wave-instructions; lane-instructions per point = x 64 / points (each
lane walks its own points); issue fraction = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8).  Clock: GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / the same
dispatch's End-Start timestamps in the GRBM pass (a kernel-trace duration from another run can
differ: the PMC program's first dispatch is cold)."""
import csv
import glob
import json
import sys
from collections import defaultdict

src = sys.argv[1]
out = sys.argv[2]
points = json.loads(sys.argv[3])   # {"k_walk<7, 2048>": points_per_dispatch, ...}
durations = json.loads(sys.argv[4]) if len(sys.argv) > 4 else {}  # kernel -> mean ns (kernel trace)
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{src}/*/run_counter_collection.csv") + glob.glob(f"{src}/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            agg[k]["_grbm_dispatch_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
res = {}
for k, d in agg.items():
    if k not in points:
        continue
    per = {c: sum(v) / len(v) for c, v in d.items()}
    p = points[k]
    e = {"counters_per_dispatch": per, "points_per_dispatch": p}
    if "TCC_EA0_RDREQ_sum" in per and "WRITE_SIZE" in per:
        wr = per["WRITE_SIZE"] * 1024
        rd_counted = per["TCC_EA0_RDREQ_sum"] * 64
        other = rd_counted - wr / 2
        e.update(hbm_read_bytes_counted_per_dispatch=rd_counted, hbm_write_bytes_per_dispatch=wr,
                 pad_read_bytes_per_dispatch=wr, probe_read_bytes_per_dispatch=other,
                 hbm_bytes_per_dispatch=other + 2 * wr,
                 hbm_bytes_per_point=(other + 2 * wr) / p, probe_read_bytes_per_point=other / p,
                 pad_bytes_per_point=2 * wr / p, uncorrected_bytes_per_point=(rd_counted + wr) / p)
    if "SQ_INSTS_VALU" in per:
        e["valu_wave_instructions_per_dispatch"] = per["SQ_INSTS_VALU"]
        e["valu_lane_instructions_per_point"] = per["SQ_INSTS_VALU"] * 64 / p
    if k in durations:
        e["kernel_trace_ns"] = durations[k]
    if "GRBM_GUI_ACTIVE" in per:
        e["grbm_dispatch_ns"] = per.pop("_grbm_dispatch_ns")
        e["effective_clock_ghz"] = per["GRBM_GUI_ACTIVE"] / 8 / e["grbm_dispatch_ns"]
        simd_cycles = 1024 * per["GRBM_GUI_ACTIVE"] / 8  # SIMD-cycles the dispatch had
        if "SQ_INSTS_VALU" in per:
            # share of the dispatch's VALU issue slots used: one wave64 instruction per SIMD per 4
            # cycles, 1024 SIMDs, GRBM_GUI_ACTIVE / 8 cycles (clock-free: both sides in cycles)
            e["valu_issue_frac"] = per["SQ_INSTS_VALU"] * 4 / simd_cycles
            # the same against the guide's 2-cycle wave64 issue (MI355X_MICROARCH.md: SIMD-32)
            e["valu_issue_frac_2cyc"] = per["SQ_INSTS_VALU"] * 2 / simd_cycles
        if "SQ_ACTIVE_INST_VALU2" in per:
            # quad-cycles in which a SIMD issued two VALU instructions (gfx950 dual issue, per SIMD)
            e["valu_dual_issue_frac"] = per["SQ_ACTIVE_INST_VALU2"] * 4 / simd_cycles
        if "SQ_WAIT_ANY" in per and "SQ_WAVE_CYCLES" in per:
            # where the waves' time goes (quad-cycles, summed over waves; disjoint per the guide)
            wc = per["SQ_WAVE_CYCLES"]
            e["wave_time_split"] = {"waiting (s_waitcnt/barrier)": per["SQ_WAIT_ANY"] / wc,
                                    "issue-stalled (dependency/pipe)": per.get("SQ_WAIT_INST_ANY", 0) / wc,
                                    "issuing": per.get("SQ_ACTIVE_INST_ANY", 0) / wc}
    if "SQ_THREAD_CYCLES_VALU" in per and "SQ_INSTS_VALU" in per:
        # thread-cycles the VALU spent per lane-instruction (class-weighted cost as the hardware counts it)
        e["valu_thread_cycles_per_instruction"] = per["SQ_THREAD_CYCLES_VALU"] / (per["SQ_INSTS_VALU"] * 64)
    res[k] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
