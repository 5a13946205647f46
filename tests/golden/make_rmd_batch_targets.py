"""Writes tests/golden/data/rmd_batch.rmd: hash160 targets for `-m rmd160 --rmd-batch-size G` with
G < 1024 (keyhunt.cpp:815-829, 3301-3307, 3349-3461).

With G < 1024 the reference's group is the first G/2 + 1 entries of its 513-entry batch inversion
(IntGroup(CPU_GRP_SIZE / 2 + 1), keyhunt.cpp:3274), the rest left zero by Int's constructor: the
product is 0, ModInv(0) is 0, so every inverse is 0 (IntGroup.cpp:36-58) and every point but the
group's centre comes out as x = -(C.x + Gn[i].x), y = -Gn[i].y (C + Gn[i] side) or +Gn[i].y
(C - Gn[i] side), with C = (key + G/2 * stride) G recomputed per group (3350-3354).  The targets:
  - the compressed hash of a group centre (a real point: found with its key),
  - the 02 hash of a "garbage" point x = -(C.x + Gn[i].x) (found: the reference reports the slot's
    key, checks the real point's hash against it and so negates it, 3619-3636),
  - the 03 hash of a group's slot 0 (x = -(C.x + Gn[G/2 - 1].x)),
  - the uncompressed hash of a garbage point (x, -Gn[i].y) (found with the slot's key, unchecked),
  - the compressed hash of an ordinary key that is no group centre (not found),
for G = 512 from 0x10000 with -n 0x100000 (chunk 0 and 1), and the same kinds for G = 1000 (whose
groups overshoot each 2^20-key chunk).  Uses the CPU oracle (test-only)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

P = 2**256 - 2**32 - 977
START, NSEQ = 0x10000, 0x100000


def garbage(g_start: int, G: int, i: int, side: int):
    """(x, y) the reference emits in the group of G keys from g_start for Gn[i] on `side` (+1: the
    C + Gn[i] point, slot G/2 + i + 1; -1: the C - Gn[i] point, slot G/2 - i - 1)."""
    cx, _ = oracle.pubkey(g_start + G // 2)
    tx, ty = oracle.pubkey(i + 1)
    x = (-(cx + tx)) % P
    return x, (P - ty) % P if side > 0 else ty


def group_start(chunk: int, g: int, G: int) -> int:
    return START + chunk * NSEQ + g * G


def rows():
    out = []
    for G in (512, 1000):
        # a centre (real point)
        k = group_start(0, 3, G) + G // 2
        x, y = oracle.pubkey(k)
        out.append(oracle.hash160_comp(x, 2 + (y & 1)))
        # 02 of a garbage point, C + Gn[10] side of group 5
        x, y = garbage(group_start(0, 5, G), G, 10, +1)
        out.append(oracle.hash160_comp(x, 2))
        # 03 of slot 0 of group 9 (C - Gn[G/2 - 1])
        x, y = garbage(group_start(0, 9, G), G, G // 2 - 1, -1)
        out.append(oracle.hash160_comp(x, 3))
        # uncompressed hash of a garbage point of chunk 1, C + Gn[20] side of group 7
        x, y = garbage(group_start(1, 7, G), G, 20, +1)
        out.append(oracle.hash160_uncomp(x, y))
        # an ordinary key that is no group centre: not found
        x, y = oracle.pubkey(group_start(0, 2, G) + 77)
        out.append(oracle.hash160_comp(x, 2 + (y & 1)))
    return out


if __name__ == "__main__":
    open(os.path.join(HERE, "data", "rmd_batch.rmd"), "w").write("\n".join(r.hex() for r in rows()) + "\n")
