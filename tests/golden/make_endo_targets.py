"""Writes tests/golden/data/endo_addr.txt and endo_x.txt: targets whose keys are lambda- or
lambda^2-multiples (and negations) of small keys in 1..2^20, so a -e scan of 1..2^20 must recover
them through the endomorphism images (keyhunt.cpp:3476-3830).  Uses the CPU oracle (test-only)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
L1 = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
L2 = L1 * L1 % N


def comp_addr(k):
    x, y = oracle.pubkey(k)
    return oracle.h160_to_address(oracle.hash160_comp(x, 2 + (y & 1)))


def uncomp_addr(k):
    x, y = oracle.pubkey(k)
    return oracle.h160_to_address(oracle.hash160_uncomp(x, y))


if __name__ == "__main__":
    addr = [comp_addr(L1 * 5 % N), comp_addr(L2 * 77 % N), comp_addr((N - L1 * 1000) % N), comp_addr((N - L2 * 31337) % N),
            uncomp_addr(L1 * 4242 % N), uncomp_addr((N - L2 * 99991) % N), uncomp_addr(N - 123456)]
    xs = ["%064x" % oracle.pubkey(k)[0] for k in (L1 * 6 % N, L2 * 888 % N, (N - L1 * 65535) % N)]
    data = os.path.join(HERE, "data")
    open(os.path.join(data, "endo_addr.txt"), "w").write("\n".join(addr) + "\n")
    open(os.path.join(data, "endo_x.txt"), "w").write("\n".join(xs) + "\n")
