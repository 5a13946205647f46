"""Summarise a round-6 placement study (tools/r06_placement.sh): per process, the BSGS walk's rate and,
for the rocprofv3 passes, each counter per giant point of k_walk<7, 2048> (every dispatch walks 2^21
lanes x one 4096-point group = 2^33 giant points), with the dispatch's duration from the kernel trace of
the same process.  Rows are sorted by rate, so a counter that separates the fast processes from the slow
ones shows as a step in its column.

usage: python tools/placement_summary.py gpurun_out/r06a OUT.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_walk<7, 2048>"
PTS = 1 << 33


def kname(s: str) -> str:
    return s.split("(")[0].replace("void ", "").strip()


def one_run(d: str) -> dict | None:
    cc = glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)
    kt = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)
    if not cc:
        return None
    per = defaultdict(lambda: defaultdict(float))   # dispatch id -> counter -> value
    for r in csv.DictReader(open(cc[0])):
        if kname(r["Kernel_Name"]) != KERNEL:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            if kname(r["Kernel_Name"]) == KERNEL:
                dur[r["Dispatch_Id"]] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    ids = sorted(per, key=int)[1:]   # the first dispatch is the warm-up call's (cold pad)
    if not ids:
        return None
    out = {"dispatches": len(ids)}
    ds = [dur[i] for i in ids if i in dur]
    if ds:
        out["ms_per_dispatch"] = 1e3 * sum(ds) / len(ds)
        out["giant_points_per_s_trace"] = PTS / (sum(ds) / len(ds))
    names = sorted({c for i in ids for c in per[i]})
    for c in names:
        v = sum(per[i][c] for i in ids) / len(ids)
        out[c + "_per_point"] = v / PTS
    if "GRBM_GUI_ACTIVE_per_point" in out and ds:
        out["clock_ghz"] = out["GRBM_GUI_ACTIVE_per_point"] * PTS / 8 / (sum(ds) / len(ds)) / 1e9
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {"source": src, "kernel": KERNEL, "giant_points_per_dispatch": PTS, "bare": [], "pmc": {}}
    bare = os.path.join(src, "bare.jsonl")
    if os.path.exists(bare):
        res["bare"] = sorted((json.loads(l) for l in open(bare) if l.strip()),
                             key=lambda r: r["giant_points_per_s_events"])
    tags = {}
    pj = os.path.join(src, "pmc.jsonl")
    if os.path.exists(pj):
        for l in open(pj):
            if l.strip():
                r = json.loads(l)
                tags[r["tag"]] = r
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        t = os.path.basename(d)
        if not os.path.isdir(d):
            continue
        r = one_run(d)
        if r is None:
            continue
        if t in tags:
            r["giant_points_per_s_events"] = tags[t]["giant_points_per_s_events"]
            r["layout"] = tags[t].get("layout")
        res["pmc"].setdefault(t.rstrip("0123456789"), []).append(dict(r, run=t))
    for k in res["pmc"]:
        res["pmc"][k].sort(key=lambda r: r.get("giant_points_per_s_trace", 0))
    json.dump(res, open(dst, "w"), indent=1)
    for r in res["bare"]:
        print("bare", r["tag"], round(r["giant_points_per_s_events"] / 1e9, 2), r.get("board"), r.get("layout"))
    for k, rows in res["pmc"].items():
        for r in rows:
            print(k, r["run"], round(r.get("giant_points_per_s_trace", 0) / 1e9, 2),
                  {c: round(v, 4) for c, v in r.items() if c.endswith("_per_point")}, round(r.get("clock_ghz", 0), 3))


if __name__ == "__main__":
    main()
