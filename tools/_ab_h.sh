set -o pipefail
O=gpurun_out/r01h; mkdir -p $O
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > $O/big.json 2> $O/big.err || { echo "bench rc=$?"; tail -20 $O/big.err; exit 1; }
KH_NO_BIG_GROUPS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > $O/small.json 2> $O/small.err || { echo "bench2 rc=$?"; tail -20 $O/small.err; exit 1; }
python - <<'P'
import json
for n in ("big","small"):
    d=json.load(open(f"gpurun_out/r01h/{n}.json")); r=d["roofline"]
    print(n, d["giant_points_per_s"]/1e9, r["mean_launch_ms"], r["giant_points_per_launch"], r["frac"], d["first_level_candidates"])
P
