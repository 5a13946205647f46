"""Interleaved in-process A/B of walk-placement variants on the bench's BSGS geometry (n = 2^44, k = 128):
for each trial, each variant frees the walk buffers (kh_release_walk), sets its environment (knobs the
engine reads when it allocates or launches: KH_PAD_SKEW, KH_BSGS_LANES, ...), then walks --calls
kh_bsgs_scan calls of --bases bases; the first call after the re-allocation is untimed.  Variants
alternate A B A B ..., so drift and the re-placement of the pad spread over all of them.

usage: python tools/env_ab.py [--trials 4] [--calls 2] [--bases 4194304] NAME:VAR=VAL[,VAR=VAL] ...
e.g.   python tools/env_ab.py base:KH_PAD_SKEW=0 skew64:KH_PAD_SKEW=64
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KH_BSGS_CALIBRATE", "0")
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--bases", type=int, default=1 << 22)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    variants = []
    for v in a.variants:
        name, _, kv = v.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        variants.append((name, env))
    keys = sorted({k for _, env in variants for k in env})
    board = bench.BoardSampler(bench.pci_bus_id(0)).start()
    e = K.Engine(0)
    info = e.bsgs_setup(1 << 44, a.k)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    two_n = 2 * info.n
    pts_call = a.bases * info.cycles * 1024
    origin, done = 1 << 124, 0
    rows = []
    for t in range(a.trials):
        for name, env in variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            e.release_walk()
            assert not e.bsgs_scan(origin + done * a.bases * two_n, a.bases)  # allocates, starts the lanes
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
            bw = board.between(b0, b1) or {}
            r = {"trial": t, "variant": name, "env": env, "giant_points_per_s_wall": a.calls * pts_call / (t1 - t0),
                 "giant_points_per_s_events": pts / (ms / 1e3), "ms_per_launch": ms / max(1, la),
                 "board": {k: bw.get(k) for k in ("board_gfxclk_mhz", "socket_power_w", "ppt_residency_frac")},
                 "layout": e.debug_layout()}
            r["points_per_joule"] = (r["giant_points_per_s_wall"] / bw["socket_power_w"]) if bw.get("socket_power_w") else None
            rows.append(r)
            print(json.dumps({"t": t, "v": name, "G": round(r["giant_points_per_s_wall"] / 1e9, 3),
                              "mhz": round(bw.get("board_gfxclk_mhz") or 0), "w": round(bw.get("socket_power_w") or 0)}),
                  file=sys.stderr, flush=True)
    board.stop()
    e.close()
    summ = {}
    for name, _ in variants:
        xs = [r["giant_points_per_s_wall"] for r in rows if r["variant"] == name]
        js = [r["points_per_joule"] for r in rows if r["variant"] == name and r["points_per_joule"]]
        summ[name] = {"mean_G": sum(xs) / len(xs) / 1e9, "min_G": min(xs) / 1e9, "max_G": max(xs) / 1e9,
                      "mean_points_per_joule": sum(js) / len(js) if js else None}
    base = variants[0][0]
    for name in summ:
        summ[name]["over_" + base] = summ[name]["mean_G"] / summ[base]["mean_G"]
    print(json.dumps({"bases_per_call": a.bases, "calls": a.calls, "trials": a.trials, "summary": summ, "rows": rows},
                     indent=1))


if __name__ == "__main__":
    main()
