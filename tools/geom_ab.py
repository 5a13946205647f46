#!/usr/bin/env python3
"""Launch-geometry A/B of the walks on one GPU (round 4): lanes per launch, groups per launch and
walk contexts in flight, each variant timed over --seconds of back-to-back calls, with the board's
clock, socket power and power-cap residency sampled meanwhile (bench.BoardSampler).

  python tools/geom_ab.py --seconds 8 > gpurun_out/geom_ab.json

Variants are "leg:lanes:groups_per_launch:contexts" (lanes / groups 0 = the engine's default).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from bench import BoardSampler  # noqa: E402

DEFAULT = ["xpoint:0:0:1", "xpoint:0:0:2", "xpoint:524288:0:1", "xpoint:1048576:1:1", "xpoint:262144:4:1",
           "rmd160:0:0:1", "rmd160:0:0:2", "rmd160:524288:0:1", "rmd160:1048576:1:1",
           "bsgs:0:0:1", "bsgs:524288:0:1"]


def run_variant(K, leg: str, lanes: int, gpl: int, ctxs: int, seconds: float, board, bsgs_bases: int = 65536) -> dict:
    engs = [K.Engine(0, lanes, gpl) for _ in range(ctxs)]
    try:
        if leg == "bsgs":
            C = bench.BSGS_CONFIGS[4]
            for e in engs:
                e.bsgs_setup(1 << 44, C["k"])
                e.bsgs_build()
                e.bsgs_set_targets([bench.decompress(C["pub"])])
            two_n = 2 * (1 << 44)
            unit_keys = two_n
            per_call = bsgs_bases
            kind = K.engine.TIME_BSGS
            origins = [(1 << 124) + i * (1 << 38) * two_n for i in range(ctxs)]
            pts_per_unit = 32768
        else:
            mode = K.KH_MODE_XPOINT if leg == "xpoint" else K.KH_MODE_ADDRESS
            row = (bench.PUZZLE63_X.to_bytes(32, "big")[:20] if leg == "xpoint"
                   else bytes.fromhex(bench.PUZZLE66_RMD))
            for e in engs:
                e.set_targets([row], bloom_items=1)
            unit_keys = bench.CHUNK
            per_call = 1
            kind = K.engine.TIME_XPOINT if leg == "xpoint" else K.engine.TIME_ADDRESS
            base = (1 << 62) if leg == "xpoint" else (1 << 65)
            origins = [base + i * (1 << 20) * bench.CHUNK for i in range(ctxs)]
            pts_per_unit = bench.CHUNK
        done = [0] * ctxs

        def call(i, e):
            o = origins[i] + done[i] * per_call * unit_keys
            if leg == "bsgs":
                assert not e.bsgs_scan(o, per_call)
            else:
                assert not e.scan(o, unit_keys, mode, K.KH_SEARCH_COMPRESS)
            done[i] += 1

        for i, e in enumerate(engs):  # warm-up: tables, lane setup
            call(i, e)
            e.synchronize()
            e.kernel_time_reset()
        stop = threading.Event()
        t0 = time.perf_counter()
        b0 = board.snapshot() if board else None

        def worker(i, e):
            while not stop.is_set():
                call(i, e)
        th = [threading.Thread(target=worker, args=(i, e)) for i, e in enumerate(engs)]
        start_calls = list(done)
        for t in th:
            t.start()
        time.sleep(seconds)
        stop.set()
        for t in th:
            t.join()
        for e in engs:
            e.synchronize()
        t1 = time.perf_counter()
        b1 = board.snapshot() if board else None
        calls = sum(d - s for d, s in zip(done, start_calls))
        la = sum(e.kernel_time(kind)[0] for e in engs)
        ms = sum(e.kernel_time(kind)[1] for e in engs)
        pts = sum(e.kernel_time(kind)[2] for e in engs)
        out = {"leg": leg, "lanes": lanes, "groups_per_launch": gpl, "contexts": ctxs, "wall_s": t1 - t0,
               "calls": calls, "points_per_s_wall": calls * per_call * pts_per_unit / (t1 - t0),
               "launches": la, "event_ms_per_launch": ms / max(la, 1), "points_per_launch": pts / max(la, 1),
               "points_per_s_events": pts / (ms / 1e3) if ms else None}
        if board:
            out["board"] = board.between(b0, b1)
        return out
    finally:
        for e in engs:
            e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--bsgs-bases", type=int, default=65536, help="bases per BSGS call (CLI: 2^35 / 32768)")
    ap.add_argument("variants", nargs="*", default=DEFAULT)
    a = ap.parse_args()
    import keyhunt_amd as K
    K.lib()
    board = BoardSampler(bench.pci_bus_id(0)).start()
    res = []
    for v in a.variants:
        leg, lanes, gpl, ctxs = v.split(":")
        r = run_variant(K, leg, int(lanes), int(gpl), int(ctxs), a.seconds, board, a.bsgs_bases)
        print(json.dumps(r), file=sys.stderr, flush=True)
        res.append(r)
    board.stop()
    print(json.dumps({"variants": res, "board_info": board.info()}, indent=1))


if __name__ == "__main__":
    main()
