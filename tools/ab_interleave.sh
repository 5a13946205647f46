#!/bin/bash
# Interleaved A/B of two library builds on ONE lease (changes under 2 % are
# judged on >= 3 A-B pairs, with their spread recorded):
#   tools/ab_interleave.sh PAIRS A B [bench.py args ...]
# A / B: "main" (keyhunt_amd/lib) or a variant of tools/build_variants.sh (variants/NAME/libkh_gpu.so).
# Runs A B A B ... (PAIRS pairs) of `bench.py --no-cpu-baseline` with short windows (override with
# bench args), then writes gpurun_out/ab/interleave_A_B.json: every run's BSGS wall / kernel rate,
# rmd160 and xpoint kernel rates, board clock and power, and per build the mean and min..max.
set -o pipefail
PAIRS=$1; A=$2; B=$3; shift 3
ARGS=${*:-"--seconds 10 --seconds-secondary 8 --steps 5 --warmup 2"}
O=gpurun_out/ab; mkdir -p $O
lib() { if [ $1 = main ]; then echo keyhunt_amd/lib/libkh_gpu.so; else echo variants/$1/libkh_gpu.so; fi; }
for i in $(seq 1 $PAIRS); do
  for v in $A $B; do
    echo "[ab] pair $i: $v" >&2
    KH_LIB=$(lib $v) timeout -k 10 240 python bench.py --no-cpu-baseline $ARGS > $O/il_${v}_$i.json 2> $O/il_${v}_$i.err \
      || { echo "bench $v pair $i rc=$?"; tail -20 $O/il_${v}_$i.err; exit 1; }
  done
done
python - $PAIRS $A $B <<'P'
import json, sys
pairs, A, B = int(sys.argv[1]), sys.argv[2], sys.argv[3]
out = {"pairs": pairs, "order": "A B A B ...", "runs": {A: [], B: []}}
for i in range(1, pairs + 1):
    for v in (A, B):
        d = json.load(open(f"gpurun_out/ab/il_{v}_{i}.json"))
        r = {"bsgs_wall_G": d["giant_points_per_s"] / 1e9, "bsgs_walk_ms": d["roofline"]["mean_launch_ms"],
             "rmd160_kernel_G": d["secondary"]["points_per_s_in_kernel"] / 1e9,
             "xpoint_kernel_G": d["tertiary"]["points_per_s_in_kernel"] / 1e9,
             "bsgs_board": d["sustained"].get("board"),
             "rmd160_board": d["secondary"]["sustained"].get("board"),
             "xpoint_board": d["tertiary"]["sustained"].get("board")}
        out["runs"][v].append(r)
summ = {}
for v in (A, B):
    s = {}
    for k in ("bsgs_wall_G", "bsgs_walk_ms", "rmd160_kernel_G", "xpoint_kernel_G"):
        xs = [r[k] for r in out["runs"][v]]
        s[k] = {"mean": sum(xs) / len(xs), "min": min(xs), "max": max(xs)}
    summ[v] = s
out["summary"] = summ
out["b_over_a"] = {k: summ[B][k]["mean"] / summ[A][k]["mean"] for k in summ[A]}
json.dump(out, open(f"gpurun_out/ab/interleave_{A}_{B}.json", "w"), indent=1)
print(json.dumps({"summary": summ, "b_over_a": out["b_over_a"]}, indent=1))
P
