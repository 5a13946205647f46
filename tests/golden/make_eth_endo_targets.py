"""Writes tests/golden/data/eth_endo.txt: Ethereum addresses of lambda- and lambda^2-multiples (and
negations) of small keys in 1..2^20, for `-m address -c eth -e` over 1..2^20.  The reference's six
images per point (keyhunt.cpp:3524-3536) are eth of P, -P, beta P, -beta P, beta P again and
-beta^2 P: lambda*k is found twice (slots 2 and 4, the second with key n - lambda^2 k), lambda^2*k is
not found at all, n - lambda^2*k is.  Uses the CPU oracle (test-only)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
L1 = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
L2 = L1 * L1 % N
KEYS = [4242, N - 123456, L1 * 5 % N, L2 * 77 % N, (N - L1 * 1000) % N, (N - L2 * 31337) % N]
# eth_endo_pair.txt: images of ONE point that hit together -- slots 2 and 3 (beta P, -beta P) of key
# 9999, so its repeated slot-4 hit must print between them and slot 5, and slots 2 and 5 (beta P,
# -beta^2 P) of key 77777 (the print order of one reference thread, `-t 1`)
PAIR_KEYS = [L1 * 9999 % N, (N - L1 * 9999) % N, L1 * 77777 % N, (N - L2 * 77777) % N]


if __name__ == "__main__":
    lines = ["0x" + oracle.eth_address(*oracle.pubkey(k)).hex() for k in KEYS]
    open(os.path.join(HERE, "data", "eth_endo.txt"), "w").write("\n".join(lines) + "\n")
    lines = ["0x" + oracle.eth_address(*oracle.pubkey(k)).hex() for k in PAIR_KEYS]
    open(os.path.join(HERE, "data", "eth_endo_pair.txt"), "w").write("\n".join(lines) + "\n")
