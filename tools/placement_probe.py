"""Does the BSGS walk's rate follow where its buffers land?  One process: per trial a spacer of a
different size is taken from the device first (torch), then either only the walk's pad is
allocated again (--mode pad: kh_release_walk, the tables stay) or the whole engine (--mode engine:
layer 1 and the pad both re-placed); each trial times --calls kh_bsgs_scan calls of --bases bases
on the bench geometry (n = 2^44, k = 128) with the board sampled meanwhile.

usage: python tools/placement_probe.py --mode pad|engine [--trials 6] [--calls 3] [--bases 4194304]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def engine():
    e = K.Engine(0)
    e.bsgs_setup(1 << 44, 128)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("pad", "engine"), required=True)
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--bases", type=int, default=1 << 22)
    a = ap.parse_args()
    board = bench.BoardSampler(bench.pci_bus_id(0)).start()
    e = engine()
    two_n = 2 * (1 << 44)
    pts_call = a.bases * 32768
    origin, done = 1 << 124, 0
    rows = []
    for t in range(a.trials):
        spacer = torch.empty((1 + 5 * t) << 30, dtype=torch.uint8, device="cuda:0")
        if a.mode == "pad":
            e.release_walk()
        else:
            e.close()
            e = engine()
        assert not e.bsgs_scan(origin + done * a.bases * two_n, a.bases)  # allocates and starts the lanes
        done += 1
        e.synchronize()
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
        del spacer
        torch.cuda.empty_cache()
        r = {"trial": t, "spacer_gb": 1 + 5 * t, "giant_points_per_s_wall": a.calls * pts_call / (t1 - t0),
             "giant_points_per_s_events": pts / (ms / 1e3), "board": board.between(b0, b1)}
        rows.append(r)
        print(json.dumps({"trial": t, "gpts": round(r["giant_points_per_s_wall"] / 1e9, 2),
                          "mhz": round(r["board"].get("board_gfxclk_mhz") or 0),
                          "w": round(r["board"].get("socket_power_w") or 0)}), file=sys.stderr, flush=True)
    board.stop()
    e.close()
    print(json.dumps({"mode": a.mode, "bases_per_call": a.bases, "calls": a.calls, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
