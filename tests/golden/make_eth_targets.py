"""Writes tests/golden/data/eth_targets.txt (0x-prefixed and bare 40-hex Ethereum addresses, the
forms forceReadFileAddressEth accepts, keyhunt.cpp:7312-7370) and eth_targets.rmd (bare hex, read
by -m rmd160 -c eth): the addresses of some keys in 1..2^20 and of one key outside that range.
Uses the CPU oracle (test-only); its Keccak is pinned by the reference's vectors (ref_vectors.json
"eth")."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

KEYS = [1, 3, 7, 8, 21, 49, 76, 224, 467, 514, 1155, 2683, 5216, 10544, 26867, 51510, 95823, 198669, 357535, 863317]
OUTSIDE = 0x1ba534 * 1000003


def eth(k):
    return oracle.eth_address(*oracle.pubkey(k)).hex()


if __name__ == "__main__":
    data = os.path.join(HERE, "data")
    lines = [("0x" if i % 2 == 0 else "") + eth(k) for i, k in enumerate(KEYS + [OUTSIDE])]
    open(os.path.join(data, "eth_targets.txt"), "w").write("\n".join(lines) + "\n")
    open(os.path.join(data, "eth_targets.rmd"), "w").write("\n".join(eth(k) for k in KEYS[::2]) + "\n")
