"""BSGS walk: giant points per pipelined round (KH_BSGS_ROUND_POINTS) and groups per launch
(kh_set_geometry's groups_per_launch) in one process, on the bench's geometry (n = 2^44, k = 128,
2^21 lanes): each variant runs --calls consecutive kh_bsgs_scan calls of --bases bases (lanes
continue across them) and reports giant points/s from the engine's walk events and the wall clock.

usage: python tools/round_ab.py [--bases 4194304] [--calls 5] [--repeat 2] VARIANT ...
VARIANT = [M x]ROUND_POINTS_LOG2:GROUPS_PER_LAUNCH, e.g. 34:2 (the default since round 5), 33:8,
3x33:3 (three groups of 2^21 lanes per launch); KH_BSGS_LANES in the environment sets the lanes
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=1 << 22)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    e = K.Engine(0)
    info = e.bsgs_setup(1 << 44, 128)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    two_n = 2 * info.n
    pts_call = a.bases * info.cycles * 1024
    origin = 1 << 124
    done = 0
    board = bench.BoardSampler(bench.pci_bus_id(0)).start()
    rows = []
    e.bsgs_scan(origin, a.bases)  # warm-up: tables resident, lanes started
    done += 1
    for rep in range(a.repeat):
        for v in a.variants:
            rp, gpl = v.split(":")
            gpl = int(gpl)
            mult, _, lg = rp.rpartition("x")        # "3x33" = 3 * 2^33 points per round
            rpts = (int(mult) if mult else 1) << int(lg)
            os.environ["KH_BSGS_ROUND_POINTS"] = str(rpts)
            e.set_geometry(0, gpl)
            e.kernel_time_reset()
            b0 = board.snapshot()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                assert not e.bsgs_scan(origin + done * a.bases * two_n, a.bases)
                done += 1
            e.synchronize()
            t1 = time.perf_counter()
            b1 = board.snapshot()
            la, ms, pts = e.kernel_time(K.engine.TIME_BSGS)
            r = {"variant": v, "repeat": rep, "round_points": rpts, "groups_per_launch": gpl,
                 "giant_points_per_s_wall": a.calls * pts_call / (t1 - t0), "giant_points_per_s_events": pts / (ms / 1e3),
                 "launches": la, "ms_per_launch": ms / la, "board": board.between(b0, b1)}
            rows.append(r)
            print(json.dumps({k: r[k] for k in ("variant", "repeat", "giant_points_per_s_wall", "ms_per_launch")}),
                  file=sys.stderr, flush=True)
    board.stop()
    e.close()
    print(json.dumps({"bases_per_call": a.bases, "calls": a.calls, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
