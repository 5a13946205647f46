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
        t = time.perf_counter()
        if name == "list":   # the same consecutive bases, handed over as a list in reverse order
            e.bsgs_scan_list([base0 + (rep * B + B - 1 - b) * two_n for b in range(B)])
        else:
            e.bsgs_scan(base0 + rep * B * two_n, B)
        e.synchronize()
        dt = time.perf_counter() - t
    out[name] = B * info.cycles * 1024 / dt / 1e9
print(json.dumps(out))
