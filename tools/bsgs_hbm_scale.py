"""BSGS with the baby-step table sized for one MI355X's 288 GB of HBM (measurement aid).

The reference's keys/s is 2M keys per giant point (M = sqrt(N) * k baby steps, keyhunt.cpp:1454-1661,
4883-4884) at a giant-point rate that, on the GPU, does not depend on the table's footprint (random
16-B probe loads run at the same rate from 64 MB to 24 GB).  So the table a GPU holds
sets its keys/s.  This builds M = 2^34 baby points (-n 2^50 -k 512: a ~185 GB blocked layer 1, the
second and third layers and the bP table, plus the 16 GB inversion pad), checks a planted key is
found, then times the bench's BSGS step (2^31 giant points) and prints one JSON line.

usage: python tools/bsgs_hbm_scale.py [LOG2_N] [K] [STEPS]   (default 50 512 6)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import keyhunt_amd as K  # noqa: E402

P = 2**256 - 2**32 - 977
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
PUZZLE125 = "0233709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e"


def ec_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0] and (p[1] + q[1]) % P == 0:
        return None
    if p == q:
        lam = 3 * p[0] * p[0] * pow(2 * p[1], P - 2, P) % P
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], P - 2, P) % P
    x = (lam * lam - p[0] - q[0]) % P
    return x, (lam * (p[0] - x) - p[1]) % P


def ec_mul(k):
    r, a = None, (GX, GY)
    while k:
        if k & 1:
            r = ec_add(r, a)
        a = ec_add(a, a)
        k >>= 1
    return r


def decompress(s):
    x = int(s[2:], 16)
    y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
    return x, (y if (y & 1) == (int(s[:2], 16) & 1) else P - y)


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    e = K.Engine(0)
    info = e.bsgs_setup(1 << log2n, k)
    tab_gb = sum(info.bloom_bytes[i] for i in range(3)) * 256 / 1e9 + info.m3 * 16 / 1e9
    print(f"N=2^{log2n} k={k}: M={info.m} (2^{info.m.bit_length() - 1}), cycles={info.cycles}, "
          f"layers+table {tab_gb:.1f} GB", file=sys.stderr, flush=True)
    t = time.perf_counter()
    e.bsgs_build()
    e.synchronize()
    build_s = time.perf_counter() - t
    print(f"build {build_s:.1f} s", file=sys.stderr, flush=True)
    two_n = 2 * info.n
    base0 = 1 << 124
    # known answer: a key inside the 8th base's window
    key = base0 + 7 * two_n + two_n // 3 + 12345
    e.bsgs_set_targets([ec_mul(key)])
    found = e.bsgs_scan(base0, 16)
    assert [f[1] for f in found] == [key], (found, hex(key))
    e.bsgs_reset_found()
    e.bsgs_set_targets([decompress(PUZZLE125)])
    B = (1 << 31) // (info.cycles * 1024)        # 2^31 giant points per step, as bench.py
    start = base0 + 64 * two_n
    e.bsgs_scan(start, B)                         # warm-up step
    e.synchronize()
    e.kernel_time_reset()
    t = time.perf_counter()
    for s in range(1, steps + 1):
        assert not e.bsgs_scan(start + s * B * two_n, B)
    e.synchronize()
    T = time.perf_counter() - t
    la, ms, pts = e.kernel_time(K.engine.TIME_BSGS)
    out = {"workload": f"-m bsgs -f 125.txt -b 125 -n 0x{1 << log2n:x} -k {k}", "M": info.m,
           "tables_gb": round(tab_gb, 1), "build_s": round(build_s, 2), "known_key_found": True,
           "steps": steps, "bases_per_step": B, "giant_points_per_s": steps * B * info.cycles * 1024 / T,
           "value_mkeys_per_s": steps * B * two_n / T / 1e6, "unit": "Mkeys/s",
           "kernel_ms_per_2^30_points": ms / pts * 2**30, "launches": la}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
