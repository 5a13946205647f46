"""The BSGS walk's two placement states inside ONE process (round 6): freeing the walk's 64-GB pad and
allocating it again alternates the walk between a fast and a slow state (profiles/r06e_pad_alloc_sweep.json).
This workload does --allocs such re-allocations on the bench geometry (n = 2^44, k = 128, 2^21 lanes);
after each, one warm-up call and --calls timed calls of 2^18 bases (one 2^33-point dispatch each).  Run
it under `rocprofv3 --pmc ... --kernel-trace`; tools/state_pmc_summary.py groups the dispatches by
allocation and sets the counters per giant point beside each allocation's walk rate.  Prints one JSON
line: the engine's own rate and the pad's address per allocation.

usage: python tools/state_pmc.py [--allocs 4] [--calls 2] [--tag NAME]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KH_BSGS_LANES", str(1 << 21))
os.environ.setdefault("KH_BSGS_CALIBRATE", "0")
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    bases = 1 << 18
    e = K.Engine(0)
    info = e.bsgs_setup(1 << 44, 128)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    two_n = 2 * info.n
    origin, done = 1 << 124, 0
    rows = []
    for k in range(a.allocs):
        e.release_walk()
        assert not e.bsgs_scan(origin + done * bases * two_n, bases)
        done += 1
        e.synchronize()
        e.kernel_time_reset()
        for _ in range(a.calls):
            assert not e.bsgs_scan(origin + done * bases * two_n, bases)
            done += 1
        e.synchronize()
        la, ms, pts = e.kernel_time(K.engine.TIME_BSGS)
        rows.append({"alloc": k, "giant_points_per_s_events": pts / (ms / 1e3), "launches": la,
                     "pad": e.debug_layout()["pad"]})
    e.close()
    print(json.dumps({"tag": a.tag, "allocs": a.allocs, "calls": a.calls, "dispatches_per_alloc": 1 + a.calls,
                      "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
