"""Summary of tools/r06_state_pmc.sh: per counter pass (one process, several pad allocations), the
k_walk<7, 2048> dispatches grouped by allocation (warm-up dispatch dropped), each allocation's walk rate
from the kernel trace and its counters per giant point (2^33 points per dispatch), then per counter the
ratio of the slow allocations' mean to the fast ones' (allocations split at the median rate).

usage: python tools/state_pmc_summary.py gpurun_out/r06f OUT.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_walk<7, 2048>"
PTS = 1 << 33


def kname(s):
    return s.split("(")[0].replace("void ", "").strip()


def one_pass(d, per_alloc):
    cc = glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)
    kt = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)
    if not cc:
        return None
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(cc[0])):
        if kname(r["Kernel_Name"]) == KERNEL:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            if kname(r["Kernel_Name"]) == KERNEL:
                dur[int(r["Dispatch_Id"])] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    ids = sorted(per)
    allocs = []
    for k in range(len(ids) // per_alloc):
        grp = ids[k * per_alloc + 1:(k + 1) * per_alloc]   # drop the warm-up dispatch
        ds = [dur[i] for i in grp if i in dur]
        row = {"alloc": k, "giant_points_per_s_trace": PTS / (sum(ds) / len(ds)) if ds else None}
        for c in sorted({c for i in grp for c in per[i]}):
            row[c + "_per_point"] = sum(per[i][c] for i in grp) / len(grp) / PTS
        if "GRBM_GUI_ACTIVE_per_point" in row and ds:
            row["clock_ghz"] = row["GRBM_GUI_ACTIVE_per_point"] * PTS / 8 / (sum(ds) / len(ds)) / 1e9
        allocs.append(row)
    rates = sorted(r["giant_points_per_s_trace"] for r in allocs)
    med = (rates[len(rates) // 2 - 1] + rates[len(rates) // 2]) / 2 if len(rates) > 1 else rates[0]
    fast = [r for r in allocs if r["giant_points_per_s_trace"] > med]
    slow = [r for r in allocs if r["giant_points_per_s_trace"] <= med]
    ratio = {}
    if fast and slow:
        for c in allocs[0]:
            if c.endswith("_per_point") or c in ("giant_points_per_s_trace", "clock_ghz"):
                f = sum(r[c] for r in fast) / len(fast)
                s = sum(r[c] for r in slow) / len(slow)
                ratio[c] = {"fast": f, "slow": s, "slow_over_fast": s / f if f else None}
    return {"allocs": allocs, "fast_vs_slow": ratio}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    meta = {}
    pj = os.path.join(src, "pmc.jsonl")
    if os.path.exists(pj):
        for l in open(pj):
            if l.strip():
                r = json.loads(l)
                meta[r["tag"]] = r
    res = {"source": src, "kernel": KERNEL, "giant_points_per_dispatch": PTS, "passes": {}}
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        if not os.path.isdir(d):
            continue
        t = os.path.basename(d)
        m = meta.get(t, {})
        r = one_pass(d, m.get("dispatches_per_alloc", 3))
        if r:
            r["engine_rows"] = m.get("rows")
            res["passes"][t] = r
    json.dump(res, open(dst, "w"), indent=1)
    for t, r in res["passes"].items():
        print(t, [round(a["giant_points_per_s_trace"] / 1e9, 2) for a in r["allocs"]])
        for c, v in r["fast_vs_slow"].items():
            print("   ", c, f"fast {v['fast']:.4g} slow {v['slow']:.4g} slow/fast {v['slow_over_fast']:.4f}")


if __name__ == "__main__":
    main()
