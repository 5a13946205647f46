"""Which buffer's placement sets the BSGS walk's state?  One process on the bench geometry (n = 2^44,
k = 128, 2^21 lanes, no calibration): for each entry of --seq, give the buffers it names fresh
allocations (kh_debug_replace: 1 layer 1, 2 the pad, 4 the lane arrays, 8 the delta tables, 16 layers
2/3, 32 a new walk stream; "r" = kh_release_walk; "s0" / "s1" = switch KH_PAD_SWZ, no move; "bN" = N ms of VALU burn first; "iN" = N ms idle first) and time --calls calls of --bases bases after one warm call.  Prints one
JSON object with every step's rate and the board's clock and power.  (Round-6 r06h ran it as
--seq 1,1,1,1,1,1,r,r,r,r.)

usage: python tools/replace_ab.py [--seq 8,8,4,4,1,1,2,2] [--calls 1] [--bases 4194304]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KH_BSGS_CALIBRATE", "0")
os.environ.setdefault("KH_BSGS_LANES", str(1 << 21))
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", default="8,8,4,4,1,1,2,2")
    ap.add_argument("--calls", type=int, default=1)
    ap.add_argument("--bases", type=int, default=1 << 22)
    a = ap.parse_args()
    board = bench.BoardSampler(bench.pci_bus_id(0)).start()
    e = K.Engine(0)
    info = e.bsgs_setup(1 << 44, 128)
    e.bsgs_build()
    e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
    two_n = 2 * info.n
    pts_call = a.bases * info.cycles * 1024
    origin, done = 1 << 124, 0
    rows = []

    def timed(what, k):
        nonlocal done
        assert not e.bsgs_scan(origin + done * a.bases * two_n, a.bases)  # warm (after a re-allocation)
        done += 1
        e.synchronize()
        b0 = board.snapshot()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            assert not e.bsgs_scan(origin + done * a.bases * two_n, a.bases)
            done += 1
        e.synchronize()
        t1 = time.perf_counter()
        bw = board.between(b0, board.snapshot()) or {}
        r = {"moved": what, "step": k, "giant_points_per_s": a.calls * pts_call / (t1 - t0),
             "mhz": bw.get("board_gfxclk_mhz"), "w": bw.get("socket_power_w"), "layout": e.debug_layout()}
        rows.append(r)
        print(json.dumps({"moved": what, "k": k, "G": round(r["giant_points_per_s"] / 1e9, 3),
                          "mhz": round(r["mhz"] or 0), "w": round(r["w"] or 0)}), file=sys.stderr, flush=True)

    names = {1: "layer1", 2: "pad", 4: "lanes", 8: "tables", 16: "layers23", 32: "stream"}
    timed("none", 0)
    for k, w in enumerate(a.seq.split(",")):
        if w == "r":
            e.release_walk()
            timed("release_walk", k)
        elif w[0] == "b":           # bN: N ms of VALU burn right before the timed calls
            e.debug_burn(float(w[1:]))
            timed("burn" + w[1:], k)
        elif w[0] == "i":           # iN: N ms idle (the board's clock rises), then the timed calls
            e.synchronize()
            time.sleep(float(w[1:]) / 1e3)
            timed("idle" + w[1:], k)
        elif w[0] in "sS":          # s0 / s1: KH_PAD_SWZ off / on (the pad's column swizzle), no move
            os.environ["KH_PAD_SWZ"] = w[1:]
            timed("swz" + w[1:], k)
        else:
            e.debug_replace(int(w))
            timed("+".join(v for b, v in names.items() if int(w) & b), k)
    board.stop()
    e.close()
    print(json.dumps({"bases_per_call": a.bases, "calls": a.calls, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
