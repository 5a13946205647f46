"""-m rmd160 --rmd-batch-size G < 1024 on the GPU (kh_set_rmd_batch, k_walk_zinv).

The reference's groups of G keys invert a partly zero IntGroup, so each group holds one real point
(its centre) and G - 1 points that are no multiples of G (keyhunt.cpp:3274, 3301-3461; see
oracle/kh_oracle.c walk_group_n).  The engine's hits are compared with the CPU oracle's restatement
(itself pinned by the reference CLI's runs, tests/test_oracle.py::test_oracle_rmd_batch_vs_reference_cli)
on targets built from centres, from those points (both sides of a group, slot 0, every hash kind)
and from ordinary keys, and the CLI runs with --rmd-batch-size against the reference CLI's own
fixtures in tests/test_gpu_scan.py (rmd160_batch*)."""
import random

import pytest

pytestmark = pytest.mark.gpu
P = 2**256 - 2**32 - 977
ORDER_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _point_rows(oracle, pts, rng):
    rows = []
    for x, y in pts:
        kind = rng.randrange(3)
        if kind == 0:
            rows.append(oracle.hash160_comp(x, 2 + (y & 1)))
        elif kind == 1:
            rows.append(oracle.hash160_comp(x, 3 - (y & 1)))
        else:
            rows.append(oracle.hash160_uncomp(x, y))
    return rows


def _targets(oracle, start, n_keys, G, rng, n=12):
    """Points the reference's walk produces in groups of G from `start`: centres, and
    x = -(C.x + (i+1)G.x) with y = -(i+1)G.y (slot G/2 + i + 1) or +(i+1)G.y (slot G/2 - i - 1)."""
    half = G // 2
    groups = (n_keys + G - 1) // G
    pts = []
    for _ in range(n):
        g = rng.randrange(groups)
        c = start + g * G + half
        t = rng.choice([0, half, G - 1, rng.randrange(G)])
        if t == half:
            pts.append(oracle.pubkey(c))
            continue
        cx, _ = oracle.pubkey(c)
        i = t - half - 1 if t > half else half - t - 1
        tx, ty = oracle.pubkey(i + 1)
        pts.append(((-(cx + tx)) % P, (P - ty) % P if t > half else ty))
    # ordinary keys (found only where they are a centre)
    pts += [oracle.pubkey(start + rng.randrange(n_keys)) for _ in range(3)]
    return _point_rows(oracle, pts, rng)


@pytest.mark.parametrize("G", [4, 8, 100, 512, 1000, 1020])
@pytest.mark.parametrize("search,endo", [(0, False), (1, False), (2, False), (2, True), (0, True)])
def test_engine_rmd_batch_vs_oracle(engine, oracle, G, search, endo):
    rng = random.Random(G * 10 + search + (5 if endo else 0))
    start = rng.getrandbits(66) | (1 << 65)
    n_keys = 1 << 15  # not a multiple of 100/1000/1020: the last group overshoots the chunk
    rows = _targets(oracle, start, n_keys, G, rng)
    engine.set_targets(rows)
    engine.set_rmd_batch(G)
    try:
        got = engine.scan(start, n_keys, mode=0, search=search, endo=endo)
    finally:
        engine.set_rmd_batch(1024)
    ref = oracle.scan_chunk(0, search, start, n_keys, rows, endo=endo, group=G)
    assert ref, "the targets should produce hits"
    assert sorted((h.key, h.compressed, h.kind) for h in got) == sorted(ref)


def test_engine_rmd_batch_1024_is_the_ordinary_walk(engine, oracle):
    rng = random.Random(3)
    start = rng.getrandbits(64)
    keys = sorted(rng.sample(range(start, start + 8192), 5))
    rows = [oracle.hash160_comp(*(lambda p: (p[0], 2 + (p[1] & 1)))(oracle.pubkey(k))) for k in keys]
    engine.set_targets(rows)
    engine.set_rmd_batch(1024)
    got = engine.scan(start, 8192, mode=0, search=0)
    assert [h.key for h in got] == keys


def test_engine_rmd_batch_refuses_bad_sizes_and_xpoint(engine, oracle):
    from keyhunt_amd.engine import KhError
    for bad in (2, 6, 1025, 2048):
        with pytest.raises(KhError):
            engine.set_rmd_batch(bad)
    engine.set_targets([bytes(20)])
    engine.set_rmd_batch(512)
    try:
        with pytest.raises(KhError):
            engine.scan(1, 4096, mode=1, search=2)
    finally:
        engine.set_rmd_batch(1024)


@pytest.mark.parametrize("G", [8, 512])
def test_engine_rmd_batch_centre_on_the_jump(engine, oracle, G):
    """A group centred on key G (start = G/2) is the lane's jump T[H] itself: the next centre is 2C,
    a doubling, which the reference gets by recomputing the centre from its key (keyhunt.cpp:3350-3354).
    Few lanes, so each walks many groups past that one."""
    rng = random.Random(G)
    start, n_keys = G // 2, 64 * G
    rows = _targets(oracle, start, n_keys, G, rng, n=24)
    engine.set_targets(rows)
    engine.set_geometry(4, 0)
    engine.set_rmd_batch(G)
    try:
        got = engine.scan(start, n_keys, mode=0, search=2)
    finally:
        engine.set_rmd_batch(1024)
        engine.set_geometry(0, 0)
    ref = oracle.scan_chunk(0, 2, start, n_keys, rows, group=G)
    assert ref
    assert sorted((h.key, h.compressed, h.kind) for h in got) == sorted(ref)


def test_engine_rmd_batch_scans_up_to_the_zero_centre(engine, oracle):
    """A chunk whose group m is centred on the key 0 mod n (the reference builds that group from its
    point at infinity, which the engine does not restate): the groups before it are scanned and their
    hits returned, with KH_E_RANGE for the rest."""
    G, m_bad = 512, 3
    start = ORDER_N - (G // 2 + m_bad * G)
    rng = random.Random(77)
    rows = _targets(oracle, start, m_bad * G, G, rng, n=16)
    engine.set_targets(rows)
    engine.set_rmd_batch(G)
    try:
        r, got = engine.scan_status(start, 8 * G, mode=0, search=2)
    finally:
        engine.set_rmd_batch(1024)
    assert r == -7  # KH_E_RANGE
    ref = oracle.scan_chunk(0, 2, start, m_bad * G, rows, group=G)
    assert ref
    assert sorted((h.key, h.compressed, h.kind) for h in got) == sorted(ref)


def test_engine_rmd_batch_near_the_order_without_a_zero_centre(engine, oracle):
    """A chunk that ends past the order but centres no group on the key 0 mod n is scanned (the old
    guard refused every chunk reaching the order): its groups below the order give the oracle's hits."""
    G = 512
    start = ORDER_N - 1000  # offset 1000 holds key 0: (1000 - 256) % 512 != 0, no group centred there
    rng = random.Random(78)
    rows = _targets(oracle, start, G, G, rng, n=8)  # the first group, wholly below the order
    engine.set_targets(rows)
    engine.set_rmd_batch(G)
    try:
        r, got = engine.scan_status(start, G, mode=0, search=2)
        r2, _ = engine.scan_status(start, 4 * G, mode=0, search=2)
    finally:
        engine.set_rmd_batch(1024)
    assert r == 0 and r2 == 0
    ref = oracle.scan_chunk(0, 2, start, G, rows, group=G)
    assert ref
    assert sorted((h.key, h.compressed, h.kind) for h in got) == sorted(ref)


def test_engine_rmd_batch_chunk_over_the_order_equals_oracle(engine, oracle):
    """The whole 4-group chunk from n - 1000: group 1 holds the key 0 mod n at a
    non-centre slot, whose zero difference would collapse a full batch inversion -- with G < 1024 every
    inverse of the reference's IntGroup is 0 anyway (oracle walk_group_n), so that group's points follow
    the same s = 0 formulas.  Targets are planted on both sides of groups 0 and 1 (and their centres);
    the engine's hits over the whole chunk, keys past the order included, equal the oracle's.  The
    oracle is pinned by the reference CLI away from the order; for keys past it (which the reference
    keeps unreduced) parity with the reference itself is unpinned: no reference fixture crosses the order
    with --rmd-batch-size."""
    G, half = 512, 256
    start = ORDER_N - 1000
    rng = random.Random(79)
    pts = []
    for off in (0, 100, 255, 256, 257, 500, 511, 512, 600, 767, 768, 769, 900, 999):
        g, t = divmod(off, G)
        c = start + g * G + half
        if t == half:
            pts.append(oracle.pubkey(c))
            continue
        cx, _ = oracle.pubkey(c)
        i = t - half - 1 if t > half else half - t - 1
        tx, ty = oracle.pubkey(i + 1)
        pts.append(((-(cx + tx)) % P, (P - ty) % P if t > half else ty))
    rows = _point_rows(oracle, pts, rng)
    engine.set_targets(rows)
    engine.set_rmd_batch(G)
    try:
        r, got = engine.scan_status(start, 4 * G, mode=0, search=2)
    finally:
        engine.set_rmd_batch(1024)
    assert r == 0
    ref = oracle.scan_chunk(0, 2, start, 4 * G, rows, group=G)
    assert len(ref) >= 8
    assert sorted((h.key, h.compressed, h.kind) for h in got) == sorted(ref)


def test_engine_rmd_batch_wrapping_stride(engine, oracle):
    """-I strides that wrap the order many times per chunk (every such chunk was
    refused).  Centres are real points: a centre planted as a target is found with its key
    start + (G/2 + m G) * stride mod n.  (Parity with the reference for keys past the order, which it
    keeps unreduced, is unpinned: no fixture holds such a run.)"""
    G = 512
    stride = (1 << 230) + 12345
    start = 0x1234567890ABCDEF
    centres = [(start + (G // 2 + m * G) * stride) % ORDER_N for m in (0, 5, 17)]
    rows = []
    for c in centres:
        x, y = oracle.pubkey(c)
        rows.append(oracle.hash160_comp(x, 2 + (y & 1)))
    engine.set_targets(rows)
    engine.set_rmd_batch(G)
    try:
        r, got = engine.scan_status(start, 32 * G, mode=0, search=0, stride=stride)
    finally:
        engine.set_rmd_batch(1024)
    assert r == 0
    assert sorted(h.key for h in got) == sorted(centres)
