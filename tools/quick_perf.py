"""Quick throughput probe of the engine (development aid; bench.py is the contract)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import keyhunt_amd as K  # noqa: E402

e = K.Engine(0)
e.set_targets([bytes.fromhex("20d45a6a762535700ce9e0b216e31994335db8a5")])
for n in (1 << 28, 1 << 32):
    e.kernel_time_reset()
    t = time.time()
    e.scan(1 << 65, n, 0, 0)
    dt = time.time() - t
    print(f"rmd160 compress {n} keys: {dt:.3f}s wall, {2 * n / dt / 1e6:.1f} Mkeys/s; walk {e.kernel_time(0)} setup {e.kernel_time(4)}", flush=True)
e.kernel_time_reset()
t = time.time()
e.scan(1 << 62, 1 << 30, 1, 2)
dt = time.time() - t
print(f"xpoint 2^30 keys: {dt:.3f}s, {(1 << 30) / dt / 1e6:.1f} Mkeys/s; walk {e.kernel_time(1)}", flush=True)
info = e.bsgs_setup(1 << 44, 128)
t = time.time()
e.bsgs_build()
print(f"bsgs k=128 build: {time.time() - t:.2f}s {e.kernel_time(3)}", flush=True)
x = int("33709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e", 16)
P = 2**256 - 2**32 - 977
y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
if y & 1:
    y = P - y
e.bsgs_set_targets([(x, y)])
for nb in (16, 128):
    e.kernel_time_reset()
    t = time.time()
    e.bsgs_scan(1 << 124, nb)
    dt = time.time() - t
    pts = nb * info.cycles * 1024
    print(f"bsgs k=128 {nb} bases: {dt:.3f}s wall, {pts / dt / 1e6:.1f} M giant pts/s = {nb * 2 * info.n / dt / 1e12:.1f} Tkeys/s "
          f"(walk {e.kernel_time(2)}, setup {e.kernel_time(4)}, cands {e.bsgs_candidates()})", flush=True)
