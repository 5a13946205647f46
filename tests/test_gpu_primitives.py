"""GPU parity of the engine's primitives against the reference-generated golden vectors
(tests/golden/ref_vectors.json, produced by the reference's own secp256k1/hash/bloom/xxhash code)
and against the CPU oracle on seeded random inputs."""
import json
import os
import random

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
P = 2**256 - 2**32 - 977
VEC = json.load(open(os.path.join(GOLDEN, "ref_vectors.json")))


def h(x):
    return int(x, 16)


def test_field_ops_vs_reference(engine):
    a = [h(v["a"]) for v in VEC["field"]]
    b = [h(v["b"]) for v in VEC["field"]]
    got = engine.field_ops(a, b)
    for v, (mul, sqr, inv, add, sub) in zip(VEC["field"], got):
        assert mul == h(v["mul"]) % P
        assert sqr == h(v["sqr"]) % P
        assert inv == h(v["inv"])
        assert add == h(v["add"]) % P
        assert sub == h(v["sub"]) % P


def test_field_ops_random(engine):
    rng = random.Random(1234)
    # carry-heavy edges: all-ones limbs in every product column and reduction position
    edges = [P - 1 - k for k in range(4)] + [2**224 - 1, 2**192 - 1, (2**256 - 1) // 3, 2**128 - 1, P - 2**128,
                                             2**255 - 1]
    a = [rng.randrange(P) for _ in range(4096)] + [0, 1, P - 1, 2**255, P - 2**32] + edges + edges[::-1]
    b = [rng.randrange(P) for _ in range(4096)] + [P - 1, P - 1, P - 1, 2**255, 2**32] + edges + edges
    # fix-ups of +-0x1000003D1 that ripple past limb 1 (the kernel's rare blocks), each pair four times
    # so it runs through the single and both paired-chain forms: a - b wraps with low 64 bits below
    # 0x1000003D1; a + b carries out of 2^256 with low 64 bits at or above 2^64 - 0x1000003D1
    ripple = [(2**64 + 7, 5 * 2**64 + 3), (0, 1), (2**64, 2**128), (P - 1, 2**255 + 0x1000003CD),
              (2**255 + 0x1000003CD, P - 1), (P - 1, P - 2**64 + 0x1000003D1 + 0x1000003D2 - 1)]
    for x, y in ripple:
        a += [x] * 4
        b += [y] * 4
    got = engine.field_ops(a, b)
    for x, y, (mul, sqr, inv, add, sub) in zip(a, b, got):
        assert mul == x * y % P
        assert sqr == x * x % P
        assert inv == (pow(x, P - 2, P) if x else 0)
        assert add == (x + y) % P
        assert sub == (x - y) % P


def test_field_mul_reduction_rare_block(engine):
    """Products that overflow each V_j / W_i slice of the device reduction (tests/_reduce_model.py),
    spread over waves whose other lanes take the fast path, and whole waves of them."""
    from _reduce_model import overflow_pairs
    rng = random.Random(99)
    pairs = overflow_pairs()
    a, b = [], []
    for k, (x, y) in enumerate(pairs):     # one rare lane per 64-lane wave, then all-rare waves
        a += [rng.randrange(P) for _ in range(63)] + [x]
        b += [rng.randrange(P) for _ in range(63)] + [y]
    a += [x for x, _ in pairs]
    b += [y for _, y in pairs]
    # squarings that overflow the slices (fe_sqr shares the reduction)
    from _reduce_model import square_overflow_inputs
    sq = square_overflow_inputs()
    for x in sq:
        a += [rng.randrange(P) for _ in range(63)] + [x]
        b += [rng.randrange(P) for _ in range(64)]
    a += sq
    b += sq
    got = engine.field_ops(a, b)
    for x, y, (mul, sqr, _inv, _add, _sub) in zip(a, b, got):
        assert mul == x * y % P
        assert sqr == x * x % P


def test_pubkeys_vs_reference(engine):
    ks = [h(v["k"]) for v in VEC["pubkeys"]]
    got = engine.pubkeys(ks)
    for v, (x, y) in zip(VEC["pubkeys"], got):
        assert x == h(v["x"]) and y == h(v["y"]), v["k"]


def test_hash160_vs_reference(engine):
    pts = [(h(v["x"]), h(v["y"])) for v in VEC["pubkeys"]]
    got = engine.hash160(pts)
    for v, (h02, h03, h04) in zip(VEC["pubkeys"], got):
        assert h02.hex() == v["h02"]
        assert h03.hex() == v["h03"]
        assert h04.hex() == v["h04"]


def test_walk_points_vs_reference(engine):
    import hashlib
    for gw in VEC["group_walk"]:
        xs, _ = engine.walk_points(h(gw["start"]), gw["n"])
        assert hashlib.sha256(xs).hexdigest() == gw["sha256_walk"]


def test_walk_points_vs_oracle_with_y(engine, oracle):
    start = 0x7CCE5EFDACC00000
    xs, ys = engine.walk_points(start, 4096, need_y=True)
    ox, oy = oracle.walk_points(start, 4, need_y=True)
    assert xs == ox and ys == oy


def test_walk_points_stride(engine, oracle):
    start, stride = 0x123456789ABCDEF, 7919
    xs, _ = engine.walk_points(start, 2048, stride=stride)
    ox, _ = oracle.walk_points(start, 2, stride=stride)
    assert xs == ox


def test_target_bloom_vs_reference(engine):
    fill = VEC["bloom_fill"]
    rows = [bytes.fromhex(x) for x in fill["items"]]
    engine.set_targets(rows, bloom_items=fill["entries"])
    import hashlib
    assert hashlib.sha256(engine.get_bloom(0)).hexdigest() == fill["sha256"]
    assert all(engine.bloom_check(0, rows))
