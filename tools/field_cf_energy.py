"""Throughput and energy of the field-arithmetic forms in tools/ubench_field_cf.hip (VERDICT round 4
item 2), on the GPU box: python tools/field_cf_energy.py [--seconds S] > gpurun_out/field_cf.json

Per variant: launches of 2^18 lanes (4 waves/SIMD), each lane a chain of ITERS dependent operations,
repeated for about S seconds; HIP events time the launches and the board's energy accumulator
(bench.BoardSampler snapshots around the launches) gives joules.  Reports operations/s, operations/J,
mean socket power and board clock, and whether each chain's canonical result equals the shipped
form's (variants 0/2, 1/3, 4/5 compute the same values mod p)."""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402  (BoardSampler)

NAMES = {0: "fe_mul (shipped, 8x32 + carry counts)", 1: "fe_sqr (shipped)", 2: "mul26 (10x26, carry-free)",
         3: "sqr26 (10x26, carry-free)", 4: "2 fe_add + 2 fe_sub (shipped)",
         5: "2 add26 + 2 sub26 + norm26 (lazy, one carry sweep)", 6: "from26 + to26 (canonical bytes)",
         7: "mul29 (9x29, carry-free)", 8: "sqr29 (9x29, carry-free)"}
OPS_PER_ITER = {0: 1, 1: 1, 2: 1, 3: 1, 4: 4, 5: 4, 6: 1, 7: 1, 8: 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--iters", type=int, default=4000)
    ap.add_argument("--lanes", type=int, default=1 << 18)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "ubench_field_cf.so"))
    lib.ub_run.restype = ctypes.c_double
    assert lib.ub_setup(ctypes.c_uint32(a.lanes)) == 0
    clock = bench.BoardSampler(None).start()
    res = {"lanes": a.lanes, "iters": a.iters, "variants": {}}
    outs = {}
    for v in range(9):
        ms1 = lib.ub_run(v, a.iters, 1)  # warm-up, and the launch time that sizes the window
        reps = max(1, int(a.seconds * 1000 / max(ms1, 1e-3)))
        s0 = clock.snapshot()
        t0 = time.perf_counter()
        ms = lib.ub_run(v, a.iters, reps)
        t1 = time.perf_counter()
        s1 = clock.snapshot()
        buf = (ctypes.c_uint32 * (a.lanes * 8))()
        lib.ub_result(buf)
        outs[v] = bytes(buf)
        ops = a.lanes * a.iters * reps * OPS_PER_ITER[v]
        b = clock.between(s0, s1) or {}
        # launches only (the snapshots bracket them within milliseconds): energy = mean power x kernel time
        joules = (b.get("socket_power_w") or 0) * (ms / 1e3)
        res["variants"][str(v)] = {"name": NAMES[v], "reps": reps, "ms": ms, "ops_per_s": ops / (ms / 1e3),
                                   "ops_per_joule": ops / joules if joules else None, "board": b}
        print(NAMES[v], f"{ops / (ms / 1e3) / 1e9:.1f} G/s", f"{b.get('socket_power_w')} W",
              f"{b.get('board_gfxclk_mhz')} MHz", file=sys.stderr, flush=True)
    clock.stop()
    res["match"] = {"mul26": outs[0] == outs[2], "sqr26": outs[1] == outs[3], "addsub26": outs[4] == outs[5],
                    "mul29": outs[0] == outs[7], "sqr29": outs[1] == outs[8]}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
