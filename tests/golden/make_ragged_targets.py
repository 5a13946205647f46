"""Write the ragged target files of the reference-CLI fixtures ragged_* (oracle/make_golden.py):
malformed lines among valid targets, to pin the reference's file-reading quirks
(forceReadFileAddress keyhunt.cpp:7239-7305, forceReadFileXPoint 7392-7490).  Targets are small
keys' addresses / public keys (keys 1..12), taken from tests/golden/data/1to32.txt and computed."""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "data")
P = 2**256 - 2**32 - 977
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)


def add(p, q):
    if p is None:
        return q
    lam = (3 * p[0] * p[0] * pow(2 * p[1], P - 2, P) if p == q else (q[1] - p[1]) * pow(q[0] - p[0], P - 2, P)) % P
    x = (lam * lam - p[0] - q[0]) % P
    return x, (lam * (p[0] - x) - p[1]) % P


def mul(k):
    r, a = None, G
    while k:
        if k & 1:
            r = add(r, a)
        a = add(a, a)
        k >>= 1
    return r


def main():
    addrs = open(os.path.join(DATA, "1to32.txt")).read().split()
    # address / rmd160 file: counted lines are those longer than 20 characters; the short line
    # consumes one count, so the last address is never read by the reference
    lines = [addrs[0], "   " + addrs[1], addrs[2] + "0", "", addrs[3],
             "# a comment that is long enough to count", addrs[4], "x" * 130, addrs[5],
             "short", addrs[6], addrs[7], addrs[8]]
    open(os.path.join(DATA, "ragged_addr.txt"), "w").write("\n".join(lines) + "\n")

    def comp(k):
        x, y = mul(k)
        return ("03" if y & 1 else "02") + f"{x:064x}"

    x5 = mul(5)[0]
    u6 = mul(6)
    # xpoint file: the first <count of 40+ character lines> lines are rows in order; "abc" takes a
    # row, so the last key's line is never read; no blank line (the reference dereferences NULL)
    lines = [comp(1), "  " + comp(2), "zz" * 21, comp(3) + "\tthree", "abc", comp(4), f"{x5:064x}",
             f"04{u6[0]:064x}{u6[1]:064x}", comp(7), comp(8)]
    open(os.path.join(DATA, "ragged_x.txt"), "w").write("\n".join(lines) + "\n")

    # BSGS public keys: first token of each 66+ character line; a wrong token length, a point off
    # the curve and an unknown prefix are refused with ParsePublicKeyHex's messages
    x_off = next(x for x in range(5, 100) if pow((x ** 3 + 7) % P, (P - 1) // 2, P) != 1)
    u7 = mul(7)
    lines = ["0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579 puzzle63", "abc",
             "ab" * 35, f"02{x_off:064x}", "05" + "11" * 32, f"04{u7[0]:064x}{u7[1]:064x}:seven"]
    open(os.path.join(DATA, "ragged_bsgs.txt"), "w").write("\n".join(lines) + "\n")
    # a digit pair sscanf("%X") cannot read: the reference exits (GetByte, SECP256K1.cpp:303-314)
    open(os.path.join(DATA, "ragged_bsgs_bad.txt"), "w").write("02" + "zz" * 32 + "\n")


if __name__ == "__main__":
    main()
