"""rmd160-only throughput probe (development aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import keyhunt_amd as K  # noqa: E402

tag = os.path.basename(os.path.dirname(os.environ.get("KH_LIB", "default/x")))
e = K.Engine(0)
rmd = bytes.fromhex("20d45a6a762535700ce9e0b216e31994335db8a5")
e.set_targets([rmd])
e.scan(1 << 65, 1 << 28, 0, 0)
for search, name in ((0, "compress"), (2, "both")):
    e.kernel_time_reset()
    t = time.time()
    n = 1 << 32 if search == 0 else 1 << 30
    e.scan(1 << 65, n, 0, search)
    dt = time.time() - t
    la, ms, pts = e.kernel_time(0)
    mult = 2 if search == 0 else 1
    print(f"[{tag}] rmd160 {name}: {mult * n / dt / 1e9:.2f} Gkeys/s wall, kernel {pts / ms / 1e6:.2f} Gpts/s", flush=True)
