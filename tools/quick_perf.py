"""Quick throughput probe of the engine (development aid; bench.py is the contract)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import keyhunt_amd as K  # noqa: E402

tag = os.environ.get("KH_LIB", "default")
e = K.Engine(0)
e.set_targets([bytes.fromhex("20d45a6a762535700ce9e0b216e31994335db8a5")])
e.scan(1 << 65, 1 << 28, 0, 0)
e.kernel_time_reset()
t = time.time()
e.scan(1 << 65, 1 << 32, 0, 0)
dt = time.time() - t
la, ms, pts = e.kernel_time(0)
print(f"[{tag}] rmd160 2^32: {2 * (1 << 32) / dt / 1e9:.2f} Gkeys/s wall, kernel {pts / ms / 1e6:.2f} Gpts/s", flush=True)
e.kernel_time_reset()
t = time.time()
e.scan(1 << 62, 1 << 31, 1, 2)
dt = time.time() - t
la, ms, pts = e.kernel_time(1)
print(f"[{tag}] xpoint 2^31: {(1 << 31) / dt / 1e9:.2f} Gkeys/s wall, kernel {pts / ms / 1e6:.2f} Gpts/s", flush=True)
x = int("33709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e", 16)
P = 2**256 - 2**32 - 977
y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
if y & 1:
    y = P - y
for layer1 in [int(v) for v in os.environ.get("KH_QP_LAYER1", "1,0").split(",")]:
    info = e.bsgs_setup(1 << 44, 128, layer1=layer1)
    t = time.time()
    e.bsgs_build()
    print(f"[{tag}] bsgs k=128 layer1={layer1} build: {time.time() - t:.2f}s", flush=True)
    e.bsgs_set_targets([(x, y)])
    e.bsgs_scan(1 << 124, 65536)
    e.kernel_time_reset()
    c0 = e.bsgs_candidates()
    t = time.time()
    e.bsgs_scan((1 << 124) + 65536 * 2 * info.n, 65536)
    dt = time.time() - t
    la, ms, pts = e.kernel_time(2)
    print(f"[{tag}] bsgs k=128 layer1={layer1} 65536 bases: wall {65536 * 32768 / dt / 1e9:.2f} G giant pts/s, "
          f"kernel {pts / ms / 1e6:.2f} Gpts/s, kernel points {pts}, candidates {e.bsgs_candidates() - c0}", flush=True)
