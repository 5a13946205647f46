"""A/B of BSGS list mode (kh_bsgs_scan_list, the -B both/random/dance path) vs continuous mode
on the bench geometry (k = 128): giant points/s of each over the same number of bases."""
import json
import sys
import time
sys.path.insert(0, ".")
import bench
import keyhunt_amd as K

e = K.Engine(0)
info = e.bsgs_setup(1 << 44, 128)
e.bsgs_build()
e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
B = 65536
two_n = 2 * info.n
base0 = 1 << 124
out = {}
for name in ("continuous", "list"):
    for rep in range(3):
        # the same consecutive bases, handed over as a list in reverse order (built before the clock)
        lst = [base0 + (rep * B + B - 1 - b) * two_n for b in range(B)] if name == "list" else None
        e.kernel_time_reset()
        t = time.perf_counter()
        if name == "list":
            e.bsgs_scan_list(lst)
        else:
            e.bsgs_scan(base0 + rep * B * two_n, B)
        e.synchronize()
        dt = time.perf_counter() - t
    la, ms, pts = e.kernel_time(K.engine.TIME_BSGS)
    out[name] = {"wall_G_pts_s": B * info.cycles * 1024 / dt / 1e9, "walk_launches": la, "walk_ms": ms,
                 "walk_G_pts_s": pts / ms / 1e6, "setup_launches": e.kernel_time(K.engine.TIME_SETUP)[0],
                 "setup_ms": e.kernel_time(K.engine.TIME_SETUP)[1]}
print(json.dumps(out))
