"""Python model of the device's 512 -> 256-bit reduction (kh_math.h fe_reduce512, KH_RED2): the
fast path (V_j / W_i multiply-adds, one carry chain, second fold) with the conditions that send a
wave to the rare block, and the rare block itself; plus operand pairs whose products overflow each
V_j / W_i (tests/test_reduce_model.py checks the model on the CPU, tests/test_gpu_primitives.py
runs the pairs through the GPU)."""
import random

P = 2**256 - 2**32 - 977
M32 = 2**32 - 1
M64 = 2**64 - 1


def _slices(T):
    t = [(T >> (32 * i)) & M32 for i in range(16)]
    full = {}
    for j in (0, 2, 4, 6):   # V_j = h_j*977 + l_j + l_{j+1} 2^32
        full[j] = t[8 + j] * 977 + (t[j] | t[j + 1] << 32)
    for i in (1, 3, 5, 7):   # W_i = h_i*977 + h_{i-1} + h_i 2^32
        full[i] = t[8 + i] * 977 + (t[7 + i] | t[8 + i] << 32)
    return full


def _chain(full):
    V = {k: v & M64 for k, v in full.items()}
    A = V[0] | V[2] << 64 | V[4] << 128 | V[6] << 192
    B = V[1] | V[3] << 64 | V[5] << 128 | V[7] << 192
    return A + (B << 32)     # limbs 0..8 and the chain's carry out of limb 8 (R9)


def fast(T):
    """(result, conditions that make the wave take the rare block)"""
    full = _slices(T)
    rare = {f"{'V' if k % 2 == 0 else 'W'}{k}" for k, v in full.items() if v >> 64}
    R = _chain(full)
    R8 = (R >> 256) & M32
    # the device tests R8 == 0, which a carry out of limb 8 (R9) implies (R8 = W7.hi + c wraps to 0)
    if R >> 288:
        assert R8 == 0
    if R8 == 0:
        rare.add("c8")
    X = R8 * 977 + (R & M64)
    if X >> 64:
        rare.add("m8")
    r1 = ((X >> 32) & M32) + R8
    r2 = ((R >> 64) & M32) + (r1 >> 32)
    if r2 >> 32:
        rare.add("c2")
    r = (((R & (2**256 - 1)) >> 96) << 96) | (r2 & M32) << 64 | (r1 & M32) << 32 | (X & M32)
    if r >> 224 == M32:
        rare.add("r7")
    return r, rare


def rare_block(T):
    """the rare block, valid for every input: lost bits back into R, then the long second fold"""
    full = _slices(T)
    m = {k: v >> 64 for k, v in full.items()}
    R = _chain(full)
    L = [(R >> (32 * q)) & M32 for q in range(10)]
    cc = 0
    for q in range(2, 9):
        s = L[q] + m[q - 2] + cc
        L[q], cc = s & M32, s >> 32
    L[9] += cc + m[7]
    h = L[8] + (L[9] << 32)
    r = [0] * 8
    v = h * 977 + L[0]
    r[0] = v & M32
    v = (v >> 32) + L[1] + (h & M32)
    r[1] = v & M32
    v = (v >> 32) + L[2] + (h >> 32)
    r[2] = v & M32
    cc = v >> 32
    for i in range(3, 8):
        s = L[i] + cc
        r[i], cc = s & M32, s >> 32
    x = sum(r[i] << (32 * i) for i in range(8))
    if cc:
        x = (x + 0x1000003D1) % 2**256
    return x - P if x >= P else x


def reduce(T):
    r, rare = fast(T)
    return rare_block(T) if rare else r


def overflow_pairs(seed=7, per=24):
    """(a, b) < p whose product overflows V_j (low limbs j, j+1 all ones, solved for a mod 2^256)
    or W_i (high limb i all ones, a = floor(T / b) for b near p), per positions 0..7"""
    rng = random.Random(seed)
    pairs = []
    for j in range(8):
        for _ in range(per):
            lo = rng.getrandbits(256) | M32 << (32 * j) | (M32 << (32 * (j + 1)) if j < 7 else 0)
            b = rng.randrange(P) | 1
            a = lo * pow(b, -1, 2**256) % 2**256
            if a < P:
                pairs.append((a, b))
    for i in range(8):
        for _ in range(per):
            th = rng.getrandbits(224) | M32 << (32 * i)
            th = min(th | M32 << 224 if i == 7 else th, P - 2**40)
            b = P - 1 - rng.getrandbits(20)
            a = ((th << 256) | (2**256 - 1)) // b
            if a < P:
                pairs.append((a, b))
    return pairs


def _sqrt_mod_2k(t, k=256):
    """a with a*a == t (mod 2^k), t odd and t == 1 (mod 8): Hensel lifting bit by bit"""
    a = 1
    for b in range(3, k):
        if (a * a - t) % (1 << (b + 1)):
            a += 1 << (b - 1)
    return a % (1 << k)


def square_overflow_inputs(seed=8, per=6):
    """a < p whose square overflows V_j (low limbs j, j+1 all ones: a square root mod 2^256, j >= 1)
    or W_i (high limb i of a^2 all ones: a = isqrt(T))"""
    import math
    rng = random.Random(seed)
    out = []
    for j in range(1, 8):
        for _ in range(per):
            lo = rng.getrandbits(256) | M32 << (32 * j) | (M32 << (32 * (j + 1)) if j < 7 else 0)
            lo = (lo & ~7) | 1   # a square mod 8
            lo &= 2**256 - 1
            a = _sqrt_mod_2k(lo)
            for c in (a, 2**256 - a):
                if c < P and (c * c) % 2**256 == lo:
                    out.append(c)
    for i in range(8):
        for _ in range(per):
            th = rng.getrandbits(224) | M32 << (32 * i)
            th = min(th | M32 << 224 if i == 7 else th, P - 2**40)
            a = math.isqrt((th << 256) | (2**256 - 1))
            if a < P:
                out.append(a)
    return out
