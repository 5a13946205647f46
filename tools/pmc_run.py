"""Small fixed workload for rocprofv3 counter passes: one BSGS launch (2^33 giant points: 2^21 lanes x
one 4096-point group, the bench's launch geometry since round 5), one
rmd160 and one xpoint launch (one 2^32-key chunk each: 2^20 lanes x one 4096-point group, the
address family's launch geometry since round 4) -- one dispatch of each dominant kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import keyhunt_amd as K  # noqa: E402

e = K.Engine(0)
info = e.bsgs_setup(1 << 44, 128)
e.bsgs_build()
e.bsgs_set_targets([bench.decompress(bench.PUZZLE125)])
e.bsgs_scan(1 << 124, 1 << 18)        # one launch: 2^21 lanes x 1 group of 4096 = 2^33 giant points
e.set_targets([bytes.fromhex(bench.PUZZLE66_RMD)], bloom_items=1)
e.scan(1 << 65, 1 << 32, K.KH_MODE_ADDRESS, K.KH_SEARCH_COMPRESS)
e.set_targets([bench.PUZZLE63_X.to_bytes(32, "big")[:20]], bloom_items=1)
e.scan(1 << 62, 1 << 32, K.KH_MODE_XPOINT, K.KH_SEARCH_COMPRESS)
e.synchronize()
print("done", e.kernel_time(2), e.kernel_time(0), e.kernel_time(1))
