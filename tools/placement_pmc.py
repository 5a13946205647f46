"""Workload for the round-6 placement study: the bench's BSGS geometry (n = 2^44,
k = 128, blocked layer 1) walked in --calls kh_bsgs_scan calls of --bases bases each at a fixed lane
count (KH_BSGS_LANES, default 2^21 here: no calibration), after one warm-up call.  Prints one JSON
line: the walk's rate from the engine's events, the board clock and power over the timed calls, and
where layer 1 and the pad landed (kh_debug_layout when the library has it).  Run it bare, or under
`rocprofv3 --pmc ... --kernel-trace` to read counters per dispatch of the same process: a process
lands in one placement state for its whole life, so each process is one sample.

usage: python tools/placement_pmc.py [--calls 4] [--bases 262144] [--k 128] [--no-board]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KH_BSGS_LANES", str(1 << 21))
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--bases", type=int, default=1 << 18)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--no-board", action="store_true")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    board = None if a.no_board else bench.BoardSampler(bench.pci_bus_id(0)).start()
    e = K.Engine(0)
    info = e.bsgs_setup(1 << 44, a.k)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    two_n = 2 * info.n
    pts_call = a.bases * info.cycles * 1024
    origin = 1 << 124
    assert not e.bsgs_scan(origin, a.bases)  # warm-up: pad allocated, lanes started
    e.synchronize()
    e.kernel_time_reset()
    b0 = board.snapshot() if board else None
    t0 = time.perf_counter()
    for c in range(a.calls):
        assert not e.bsgs_scan(origin + (c + 1) * a.bases * two_n, a.bases)
    e.synchronize()
    t1 = time.perf_counter()
    b1 = board.snapshot() if board else None
    la, ms, pts = e.kernel_time(K.engine.TIME_BSGS)
    out = {"tag": a.tag, "pid": os.getpid(), "k": a.k, "lanes": int(os.environ["KH_BSGS_LANES"]),
           "calls": a.calls, "bases_per_call": a.bases, "launches": la,
           "giant_points_per_s_events": pts / (ms / 1e3), "giant_points_per_s_wall": a.calls * pts_call / (t1 - t0),
           "ms_per_launch": ms / max(1, la)}
    if board:
        bw = board.between(b0, b1)
        out["board"] = {k: bw.get(k) for k in ("board_gfxclk_mhz", "socket_power_w", "ppt_residency_frac",
                                                "average_umc_activity") if k in bw}
        board.stop()
    lay = e.debug_layout() if hasattr(e, "debug_layout") else None
    if lay:
        out["layout"] = lay
    e.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
