"""BSGS giant-step throughput vs k (layer-1 footprint) and layout (development aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import keyhunt_amd as K  # noqa: E402

x = int("33709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e", 16)
P = 2**256 - 2**32 - 977
y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
e = K.Engine(0)
for k, layer1 in [(int(a), int(b)) for a, b in (s.split(":") for s in sys.argv[1:])]:
    info = e.bsgs_setup(1 << 44, k, layer1=layer1)
    e.bsgs_build()
    e.bsgs_set_targets([(x, y)])
    bases = max(1, (1 << 31) // (info.cycles * 1024))
    e.bsgs_scan(1 << 124, bases)
    e.kernel_time_reset()
    t = time.time()
    e.bsgs_scan((1 << 124) + bases * 2 * info.n, bases)
    dt = time.time() - t
    la, ms, pts = e.kernel_time(2)
    print(f"k={k} layer1={layer1} layer1 MB={256 * info.bloom_bytes[0] / 2**20:.0f}: kernel {pts / ms / 1e6:.2f} G pts/s, "
          f"wall {bases * info.cycles * 1024 / dt / 1e9:.2f}", flush=True)
