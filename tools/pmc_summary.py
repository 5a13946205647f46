"""Aggregate rocprofv3 --pmc passes (gpurun_out/pmc*/<pass>/run_counter_collection.csv) into a per-kernel
summary: counters per dispatch and per point.  Corrections (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE is TCC_EA0_RDREQ x 64 B (KB units); we report read bytes = TCC_EA0_RDREQ x 64 B and write
bytes = WRITE_SIZE x 1024 B.  Both are per dispatch of the profiled geometry."""
import csv
import glob
import json
import sys
from collections import defaultdict

src = sys.argv[1]
out = sys.argv[2]
points = json.loads(sys.argv[3])   # {"k_walk<4>": points_per_dispatch, ...}
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{src}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, d in agg.items():
    if k not in points:
        continue
    per = {c: sum(v) / len(v) for c, v in d.items()}
    p = points[k]
    e = {"counters_per_dispatch": per, "points_per_dispatch": p}
    if "TCC_EA0_RDREQ_sum" in per:
        e["hbm_read_bytes_per_dispatch"] = per["TCC_EA0_RDREQ_sum"] * 64
    if "WRITE_SIZE" in per:
        e["hbm_write_bytes_per_dispatch"] = per["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_per_dispatch" in e and "hbm_write_bytes_per_dispatch" in e:
        e["hbm_bytes_per_point"] = (e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]) / p
    if "SQ_INSTS_VALU" in per:
        e["valu_lane_instructions_per_point"] = per["SQ_INSTS_VALU"] * 64 / p
    res[k] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
