"""Where a BSGS list call's time goes: host wall clock per kh_bsgs_scan_list / kh_bsgs_scan call
against the engine's own kernel timers (walk = kind 2, lane setup = kind 4), on the CLI's call
geometry (bench config: n = 2^44, k = 128, 2^20 bases of 32768 giant points per call).

usage: python tools/bsgs_list_probe.py [--calls 4] [--bases 1048576] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keyhunt_amd import Engine  # noqa: E402
from keyhunt_amd.engine import KhBsgsFound, be32, lib  # noqa: E402


def one_call(e, rng, mode, n_bases, out, nf):
    if mode == "list":
        raw = rng.integers(0, 256, size=(n_bases, 32), dtype=np.uint8)
        raw[:, :16] = 0
        raw[:, 16] &= 0x1F                      # 125-bit bases
        buf = raw.tobytes()
    else:
        start = int(rng.integers(1, 1 << 62)) << 60
    e.kernel_time_reset()
    t0 = time.perf_counter()
    if mode == "list":
        r = lib().kh_bsgs_scan_list(e._ctx, buf, n_bases, out, 4, ctypes.byref(nf))
    else:
        r = lib().kh_bsgs_scan(e._ctx, be32(start), n_bases, out, 4, ctypes.byref(nf))
    wall = (time.perf_counter() - t0) * 1e3
    assert r == 0, r
    walk_n, walk_ms, pts = e.kernel_time(2)
    _, setup_ms, lanes = e.kernel_time(4)
    return {"mode": mode, "wall_ms": round(wall, 2), "walk_ms": round(walk_ms, 2), "walk_launches": walk_n,
            "setup_ms": round(setup_ms, 2), "points": pts, "setup_lanes": lanes,
            "gpu_frac": round((walk_ms + setup_ms) / wall, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--bases", type=int, default=1 << 20)
    ap.add_argument("--geom", default="0:0", help="comma list of lanes:groups_per_launch (0 = default)")
    ap.add_argument("--modes", default="list,progression")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    e = Engine(0)
    p = e.bsgs_setup(1 << 44, 128)
    e.bsgs_build()
    # a target outside every scanned window (pubkey of 1: no 125-bit base reaches it)
    e.bsgs_set_targets([(0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
                         0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)])
    out = (KhBsgsFound * 4)()
    nf = ctypes.c_uint32(0)
    rows = []
    for geom in a.geom.split(","):
        g_lanes, g_launch = (int(x) for x in geom.split(":"))
        e.set_geometry(g_lanes, g_launch)
        for mode in a.modes.split(","):
            for c in range(a.calls):
                rows.append(one_call(e, rng, mode, a.bases, out, nf))
                rows[-1].update(geom=geom, call=c)
                print(json.dumps(rows[-1]), flush=True)
    e.close()
    res = {"config": {"n": 1 << 44, "k": 128, "bases_per_call": a.bases, "giant_points_per_base": p.cycles * 1024},
           "calls": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
