"""Write the target files of the near-order reference-CLI fixtures (oracle/make_golden.py,
*_near_order): keys within 2^20 of the group order n, whose points are the negations of small
keys' points.  Test infrastructure: uses the CPU oracle's hash160."""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "data")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle  # noqa: E402

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


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


def address(h160: bytes) -> str:
    d = b"\x00" + h160
    d += hashlib.sha256(hashlib.sha256(d).digest()).digest()[:4]
    v = int.from_bytes(d, "big")
    s = ""
    while v:
        v, r = divmod(v, 58)
        s = B58[r] + s
    return "1" * (len(d) - len(d.lstrip(b"\x00"))) + s


def h160(k):
    x, y = mul(k)
    return oracle.hash160_comp(x, 3 if y & 1 else 2)


def main():
    keys = [N - 1, N - 0x1234, N - 0xABCDE]
    lines = [address(h160(k)) for k in keys] + [h160(N - 2).hex()]
    open(os.path.join(DATA, "near_order_addr.txt"), "w").write("\n".join(lines) + "\n")
    lines = []
    for k in (5, 0x1000, 0xFFFFF):
        x, y = mul(k)
        lines.append(("03" if y & 1 else "02") + f"{x:064x}")
    open(os.path.join(DATA, "near_order_x.txt"), "w").write("\n".join(lines) + "\n")
    print(f"window {N - 0x100000:x}:{N - 1:x}")


if __name__ == "__main__":
    main()
