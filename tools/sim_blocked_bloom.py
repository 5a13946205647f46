"""False-positive rate of blocked layer-1 bloom layouts: Poisson model vs simulation (development aid).

python tools/sim_blocked_bloom.py  -> prints, per bit-budget multiplier, the model FP and the simulated
FP of (a) double hashing inside the 512-bit block (the rejected draft) and (b) the LCG positions
the engine uses (kh_kernels.h).  Items and queries are uniform 64-bit hashes a."""
import math

import numpy as np

BPE = 28.7551   # bits per entry of bloom_init2(., 1e-6), bloom/bloom.cpp:163-176
MUL, ADD = 0x9E3779B1, 0x7F4A7C15


def model(lam: float, k: int, bb: int = 512) -> float:
    s, p = 0.0, math.exp(-lam)
    for n in range(0, 400):
        if n:
            p *= lam / n
        s += p * (1 - math.exp(-k * n / bb)) ** k
    return s


def positions(a: np.ndarray, k: int, scheme: str):
    if scheme == "double":
        g1 = ((a >> np.uint64(41)) & np.uint64(511)).astype(np.int64)
        g2 = (((a >> np.uint64(50)) & np.uint64(511)) | np.uint64(1)).astype(np.int64)
        return [(g1 + i * g2) & 511 for i in range(k)]
    s = (a >> np.uint64(32)).astype(np.uint64)
    out = []
    for _ in range(k):
        s = (s * np.uint64(MUL) + np.uint64(ADD)) & np.uint64(0xFFFFFFFF)
        out.append((s >> np.uint64(23)).astype(np.int64))
    return out


def simulate(items: int, mult: float, k: int, scheme: str, queries: int = 3_000_000, seed: int = 1) -> float:
    rng = np.random.default_rng(seed)
    blocks = math.ceil(math.ceil(items * BPE) * mult / 512)
    filt = np.zeros((blocks, 512), dtype=bool)
    a = rng.integers(0, 2**64 - 1, size=items, dtype=np.uint64)
    blk = (a % np.uint64(blocks)).astype(np.int64)
    for p in positions(a, k, scheme):
        filt[blk, p] = True
    q = rng.integers(0, 2**64 - 1, size=queries, dtype=np.uint64)
    blk = (q % np.uint64(blocks)).astype(np.int64)
    ok = np.ones(queries, dtype=bool)
    for p in positions(q, k, scheme):
        ok &= filt[blk, p]
    return float(ok.mean())


if __name__ == "__main__":
    items = 32768
    print(f"reference layout (unblocked) design FP: {(1 - math.exp(-20 / BPE)) ** 20:.3g}")
    for mult in (1.0, 1.5, 2.0):
        lam = 512 / (BPE * mult)
        print(f"bits x{mult}: model {model(lam, 20):.3g}  double-hash sim {simulate(items, mult, 20, 'double'):.3g}"
              f"  LCG sim {simulate(items, mult, 20, 'lcg'):.3g}")


def split128_masks(a: np.ndarray):
    """Masks of the split-block layout (kh_kernels.h): 4 words x 4 bits from LCG fields."""
    s = (a >> np.uint64(32)).astype(np.uint64)
    fields = []
    for _ in range(6):
        s = (s * np.uint64(MUL) + np.uint64(ADD)) & np.uint64(0xFFFFFFFF)
        fields += [(s >> np.uint64(27)), (s >> np.uint64(22)) & np.uint64(31), (s >> np.uint64(17)) & np.uint64(31)]
    masks = []
    for w in range(4):
        m = np.zeros_like(s)
        for j in range(4):
            m |= np.uint64(1) << fields[4 * w + j]
        masks.append(m)
    return masks


def simulate_split128(items: int, mult: float, queries: int = 4_000_000, seed: int = 2) -> float:
    rng = np.random.default_rng(seed)
    blocks = math.ceil(math.ceil(items * BPE) * mult / 128)
    filt = np.zeros((blocks, 4), dtype=np.uint64)
    a = rng.integers(0, 2**64 - 1, size=items, dtype=np.uint64)
    blk = (a % np.uint64(blocks)).astype(np.int64)
    for w, m in enumerate(split128_masks(a)):
        np.bitwise_or.at(filt[:, w], blk, m)
    q = rng.integers(0, 2**64 - 1, size=queries, dtype=np.uint64)
    blk = (q % np.uint64(blocks)).astype(np.int64)
    ok = np.ones(queries, dtype=bool)
    for w, m in enumerate(split128_masks(q)):
        ok &= (filt[blk, w] & m) == m
    return float(ok.mean())


def model_split(lam: float, words: int = 4, wbits: int = 32, per_word: int = 4) -> float:
    s, p = 0.0, math.exp(-lam)
    for n in range(0, 400):
        if n:
            p *= lam / n
        s += p * (1 - (1 - 1 / wbits) ** (n * per_word)) ** (words * per_word)
    return s


if __name__ == "__main__":
    for mult in (2.0, 3.0):
        print(f"split-block 128 (4 words x 4 bits), bits x{mult}: model {model_split(128 / (BPE * mult)):.3g}"
              f"  sim {simulate_split128(65536, mult):.3g}")


def pk128_masks(s0: np.ndarray, s1: np.ndarray):
    """Masks of the packed-shift layout (kh_kernels.h kh_blk_masks, KH_PK_MASKS): word w gets, from
    s = s_{w/2}, a = s >> 8*(w%2) and b = a >> 4, bits a & 15, 16 + (a >> 16 & 15), b & 15, 16 + (b >> 16 & 15)."""
    masks = []
    for w in range(4):
        a = (s0 if w < 2 else s1) >> np.uint64(8 * (w % 2))
        m = np.zeros_like(a)
        for v in (a, a >> np.uint64(4)):
            m |= np.uint64(1) << (v & np.uint64(15))
            m |= np.uint64(1) << (np.uint64(16) + ((v >> np.uint64(16)) & np.uint64(15)))
        masks.append(m)
    return masks


def simulate_pk128(items: int, mult: float, queries: int = 4_000_000, seed: int = 3) -> float:
    rng = np.random.default_rng(seed)
    blocks = math.ceil(math.ceil(items * BPE) * mult / 128)
    filt = np.zeros((blocks, 4), dtype=np.uint64)

    def draw(n):
        return (rng.integers(0, blocks, size=n), rng.integers(0, 2**32, size=n, dtype=np.uint64),
                rng.integers(0, 2**32, size=n, dtype=np.uint64))
    blk, s0, s1 = draw(items)
    for w, m in enumerate(pk128_masks(s0, s1)):
        np.bitwise_or.at(filt[:, w], blk, m)
    blk, s0, s1 = draw(queries)
    ok = np.ones(queries, dtype=bool)
    for w, m in enumerate(pk128_masks(s0, s1)):
        ok &= (filt[blk, w] & m) == m
    return float(ok.mean())


if __name__ == "__main__":
    lam = 128 / (BPE * 3.0)
    print(f"packed-shift split-block 128 (8 halves x 2 bits), bits x3.0: model "
          f"{model_split(lam, words=8, wbits=16, per_word=2):.3g}  sim {simulate_pk128(65536, 3.0):.3g}")
