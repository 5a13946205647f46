"""BSGS parity on the GPU: baby-step tables (three bloom layers + sorted bP table) bit-identical to
the reference's at small M (tests/golden/ref_vectors.json), first-level candidates (base, giant
index) and their layer-2 masks identical to the CPU oracle's, and found keys identical to the reference CLI on known-answer windows
(tests/golden/ref_e2e.json), including the benchmark configuration (k = 128)."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN
from _cli import check_against_reference, run_cli, without_threads

pytestmark = pytest.mark.gpu
VEC = json.load(open(os.path.join(GOLDEN, "ref_vectors.json")))
E2E = json.load(open(os.path.join(GOLDEN, "ref_e2e.json")))


@pytest.mark.parametrize("cfg", VEC["bsgs_build"], ids=lambda c: f"n{c['n']:x}_k{c['k']}")
def test_baby_tables_match_reference(engine, cfg):
    info = engine.bsgs_setup(cfg["n"], cfg["k"], layer1=0)   # KH_LAYER1_REFERENCE: bit-identical tables
    assert (info.m, info.m2, info.m3) == (cfg["m"], cfg["m2"], cfg["m3"])
    assert list(info.bloom_bytes) == cfg["bytes"]
    engine.bsgs_build()
    for layer, key in ((1, "sha256_l1"), (2, "sha256_l2"), (3, "sha256_l3")):
        assert hashlib.sha256(engine.get_bloom(layer)).hexdigest() == cfg[key], layer
    assert hashlib.sha256(engine.get_bsgs_table()).hexdigest() == cfg["sha256_table"]


@pytest.mark.parametrize("n,k", [(1 << 22, 2), (1 << 24, 3)], ids=["k2_continuous", "k3_overlapping_bases"])
def test_candidates_and_key_vs_oracle(engine, oracle, n, k):
    """k = 3 is the non-power-of-two case: cycles*1024 > aux, bases overlap (SURVEY 8a note 13)."""
    p = oracle.bsgs_params(n, k)
    tabs = oracle.BsgsTables(p)
    engine.bsgs_setup(n, k, layer1=0)
    engine.bsgs_build()
    assert engine.get_bloom(1) == tabs.bf1.raw
    assert engine.get_bloom(2) == tabs.bf2.raw
    assert engine.get_bloom(3) == tabs.bf3.raw
    assert engine.get_bsgs_table() == tabs.table_bytes()
    key = 0x5A5A5A5A123456
    q = oracle.pubkey(key)
    # the key sits near the END of the 4th base (beyond the 3rd base's overlap when k = 3)
    start = key - 4 * 2 * p.n + 12345
    # no hit in the first 3 bases: the same first-level candidates as the oracle; found in the 4th
    engine.bsgs_set_targets([q])
    c0 = engine.bsgs_candidates()
    engine.bsgs_log_candidates(True)
    assert engine.bsgs_scan(start, 3) == []
    got = sorted((b, a) for b, a, _ in engine.bsgs_logged_candidates())
    engine.bsgs_log_candidates(False)
    okey, ocands = tabs.scan(start, 3, q)
    # the same first-level candidates (base, giant index), not only as many
    assert okey is None and engine.bsgs_candidates() - c0 == len(ocands) and got == ocands
    found = engine.bsgs_scan(start + 3 * 2 * p.n, 1)
    assert found == [(0, key)]
    okey, _ = tabs.scan(start, 4, q)
    assert okey == key


def test_candidate_list_and_masks_vs_oracle(engine, oracle):
    """Full-fill layers (M/256 = 16384 entries per shard, past the 10000-entry floor, so layer 1
    has the reference's 1e-6 false-positive rate): over 4000 bases (4.1M giant points) the engine's
    first-level candidates -- (base, giant index a), keyhunt.cpp:4819-4823 -- are exactly the
    oracle's sequential worker's, false positives included, and each one's layer-2 mask equals the
    oracle's bsgs_secondcheck (keyhunt.cpp:5151-5184).  The engine's tables are first checked
    byte-identical to the reference's (tests/golden/ref_tables.json's n100000000_k64 digests via
    their raw shards), then handed to the oracle's scan."""
    import hashlib
    n, k, nb = 1 << 32, 64, 4000
    p = oracle.bsgs_params(n, k)
    engine.bsgs_setup(n, k, layer1=0)
    engine.bsgs_build()
    raw = [engine.get_bloom(1), engine.get_bloom(2), engine.get_bloom(3), engine.get_bsgs_table()]
    tabs = oracle.BsgsTables.from_raw(p, *raw)
    key = 0x5A5A5A5A123456
    q = oracle.pubkey(key)
    start = key - nb * 2 * p.n + 12345        # the key lies in the last base
    okey, ocands = tabs.scan(start, nb, q)
    assert okey == key and len(ocands) >= 3   # false positives and the true candidate
    engine.bsgs_set_targets([q])
    engine.bsgs_log_candidates(True)
    assert engine.bsgs_scan(start, nb) == [(0, key)]
    got = engine.bsgs_logged_candidates()
    engine.bsgs_log_candidates(False)
    got = sorted(got)
    # the engine walks whole rounds: compare up to the oracle's last candidate (the true one)
    assert [(b, a) for b, a, _ in got][: len(ocands)] == ocands
    omask = oracle.bsgs_second_masks(tabs, [start + b * 2 * p.n + a * 2 * p.m for b, a in ocands], q)
    assert [m for _, _, m in got[: len(ocands)]] == omask
    assert omask[-1] != 0 and all(m == 0 for m in omask[:-1])
    # the bP rows the oracle used are the reference's: the .tbl file the reference CLI wrote at this
    # (n, k) is the rows then their sha256 (tests/golden/ref_tables.json); the three layers are
    # compared file for file with the reference's in tests/test_gpu_tables.py
    ref = json.load(open(os.path.join(GOLDEN, "ref_tables.json")))["n100000000_k64"]["files"]
    tbl = raw[3] + hashlib.sha256(raw[3]).digest()
    assert hashlib.sha256(tbl).hexdigest() == ref[f"keyhunt_bsgs_2_{p.m3}.tbl"]


def test_blocked_layer1_candidate_list_vs_oracle(engine, oracle):
    """The shipped layer-1 layout (blocked, the engine's own) on the same footing as the reference
    layout above: over 8000 bases (8.2M giant points) the engine's first-level candidates are
    exactly those of the oracle's sequential worker probing the blocked layout by its specification
    (oracle/kh_oracle.c or_blk_check), false positives included, and each one's layer-2 mask equals
    the oracle's bsgs_secondcheck.  Layer 1 is handed over as the engine built it (its bytes are
    pinned to the specification by test_blocked_layer1_bytes_match_layout_spec); layers 2-3 and the
    bP rows are the reference layout."""
    n, k, nb = 1 << 32, 64, 8000
    p = oracle.bsgs_params(n, k)
    info = engine.bsgs_setup(n, k, layer1=1)
    assert info.layer1_layout == 1
    blocks = info.bloom_bits[0] // 128
    engine.bsgs_build()
    raw = [engine.get_bloom(1), engine.get_bloom(2), engine.get_bloom(3), engine.get_bsgs_table()]
    assert len(raw[0]) == 256 * 16 * blocks
    tabs = oracle.BsgsTables.from_raw(p, *raw, l1_blocks=blocks)
    key = 0x5A5A5A5A123456
    q = oracle.pubkey(key)
    start = key - nb * 2 * p.n + 12345        # the key lies in the last base
    okey, ocands = tabs.scan(start, nb, q)
    assert okey == key and len(ocands) >= 2   # false positives and the true candidate
    engine.bsgs_set_targets([q])
    engine.bsgs_log_candidates(True)
    assert engine.bsgs_scan(start, nb) == [(0, key)]
    got = sorted(engine.bsgs_logged_candidates())
    engine.bsgs_log_candidates(False)
    assert [(b, a) for b, a, _ in got][: len(ocands)] == ocands
    omask = oracle.bsgs_second_masks(tabs, [start + b * 2 * p.n + a * 2 * p.m for b, a in ocands], q)
    assert [m for _, _, m in got[: len(ocands)]] == omask


BSGS_CASES = [k for k in E2E if k.startswith("bsgs")]
SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


@pytest.mark.parametrize("name", BSGS_CASES)
def test_cli_bsgs_matches_reference(name):
    """Found keys (file records and the stdout lines, keyhunt.cpp:4825-4840) equal the reference
    CLI's; each distinct hit once (overlapping GGSB bases let several reference threads print the
    same key before the exit)."""
    ref = E2E[name]
    check_against_reference(ref, without_threads(ref["argv"]), name)


def test_bench_config_k128_known_answer():
    """configs[3] geometry (-k 128, N = 2^44, M = 2^29: 1.84 GB layer-1 bloom) on a window that holds
    puzzle 125's key (verified by the reference)."""
    p, hits = run_cli(["-m", "bsgs", "-f", "125.txt", "-k", "128", "-r",
                       "1c533b6bb7f0804e0995fe0000000000:1c533b6bb7f0804e09963e0000000000"], timeout=900)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert [h["key"] for h in hits] == ["1c533b6bb7f0804e09960225e44877ac"]


def test_cli_first_call_calibrates_and_finds_the_key():
    """The CLI's first 2^35-point call (2^20 bases at k = 128) holds the placement calibration's four
    parts; puzzle 125's key placed in the third part (2^19 + 1000 bases after the range start) is found,
    the same key as in the reference-verified window above."""
    start = 0x1c533b6bb7f0804e0995fe0000000000 - ((1 << 19) + 1000) * (1 << 45)
    end = start + (1 << 20) * (1 << 45)
    p, hits = run_cli(["-m", "bsgs", "-f", "125.txt", "-k", "128", "-r", f"{start:x}:{end:x}"], timeout=900)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert [h["key"] for h in hits] == ["1c533b6bb7f0804e09960225e44877ac"]


def test_cli_two_contexts_calibrate_and_find_the_key():
    """-g 2 on one GPU over two calls' worth of bases: each context's first 2^35-point call calibrates
    (each holds its own 2^21-lane pad), and the key, placed in the second call, is found once."""
    start = 0x1c533b6bb7f0804e0995fe0000000000 - ((1 << 20) + (1 << 19) + 77) * (1 << 45)
    end = start + (1 << 21) * (1 << 45)
    p, hits = run_cli(["-m", "bsgs", "-f", "125.txt", "-k", "128", "-g", "2", "-r", f"{start:x}:{end:x}"],
                      timeout=900)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert sorted({h["key"] for h in hits}) == ["1c533b6bb7f0804e09960225e44877ac"]


def test_config5_geometry_k512_known_answer():
    """configs[4] geometry (-k 512: M = 2^31, 7.36 GB layer-1 bloom per GPU) on the window that holds
    puzzle 130's key (verified by the reference)."""
    p, hits = run_cli(["-m", "bsgs", "-f", "130.txt", "-k", "512", "-r",
                       "33e7665705359f04f28b8880000000000:33e7665705359f04f28b8c80000000000"], timeout=900)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert [h["key"] for h in hits] == ["33e7665705359f04f28b88cf897c603c9"]


def test_bsgs_multi_target_and_not_found(engine, oracle):
    """Several targets in one scan (the reference loops all targets per base); keys outside the
    scanned bases are not reported; kh_bsgs_reset_found re-arms targets."""
    n, k = 1 << 24, 4
    engine.bsgs_setup(n, k, layer1=1)
    engine.bsgs_build()
    p = oracle.bsgs_params(n, k)
    start = 0x10000000000
    keys = [start + 5, start + 3 * 2 * p.n + 1000, start + 40 * 2 * p.n]  # bases 0, 3 and (outside) 40
    engine.bsgs_set_targets([oracle.pubkey(x) for x in keys])
    found = sorted(engine.bsgs_scan(start, 8))
    assert found == [(0, keys[0]), (1, keys[1])]
    assert engine.bsgs_scan(start, 8) == []          # already found: skipped like bsgs_found[]
    engine.bsgs_reset_found()
    assert sorted(engine.bsgs_scan(start, 8)) == found


@pytest.mark.parametrize("layer1", [0, 1], ids=["reference", "blocked"])
def test_layer1_layouts_no_false_negative_and_fp_rate(engine, oracle, layer1):
    """Every baby X is in layer 1 (bloom has no false negatives) in both layouts; random X's pass at
    a rate near the design error (reference 1e-6, blocked 6.6e-7)."""
    import random
    n, k = 1 << 30, 8                       # M = 2^18 babies
    info = engine.bsgs_setup(n, k, layer1=layer1)
    assert info.layer1_layout == layer1
    engine.bsgs_build()
    babies = [oracle.pubkey(i + 1)[0].to_bytes(32, "big") for i in range(0, info.m, info.m // 512)]
    assert all(engine.bloom_check(1, babies))
    rng = random.Random(11)
    rnd = [rng.getrandbits(256).to_bytes(32, "big") for _ in range(200000)]
    fp = sum(engine.bloom_check(1, rnd))
    assert fp <= 5   # expectation 0.2 (reference) / 0.13 (blocked) false positives


def test_blocked_and_reference_find_same_keys(engine, oracle):
    """Found keys do not depend on the layer-1 layout (refinement uses layers 2/3 + table)."""
    n, k = 1 << 26, 8
    key = 0x3A5F0C3D2B1E00 + 12345
    results = []
    for layer1 in (0, 1):
        p = engine.bsgs_setup(n, k, layer1=layer1)
        engine.bsgs_build()
        engine.bsgs_set_targets([oracle.pubkey(key)])
        start = key - 7 * 2 * p.n - 999
        results.append(engine.bsgs_scan(start, 16))
    assert results[0] == results[1] == [(0, key)]


def test_blocked_layer1_bytes_match_layout_spec(engine, oracle):
    """The blocked (split-block) layer-1 bloom is bit-exact with its specification (kh_kernels.h
    kh_blk_masks): shard X[0]; 16-byte block (u * blocks) >> 32 with u = X[8..12); four little-endian
    u32 words; word w gets, from s = s_{w/2} (big-endian u32s s0 = X[12..16), s1 = X[16..20)),
    a = s >> 8*(w%2) and b = a >> 4, the bits a & 15, 16 + ((a >> 16) & 15), b & 15 and
    16 + ((b >> 16) & 15) (two per 16-bit half: one v_pk_lshlrev_b16 per pair)."""
    info = engine.bsgs_setup(1 << 20, 1, layer1=1)       # M = 1024 babies
    engine.bsgs_build()
    blocks = info.bloom_bits[0] // 128
    assert info.bloom_bytes[0] == blocks * 16 and info.bloom_hashes[0] == 16
    model = bytearray(256 * blocks * 16)
    for i in range(1, info.m + 1):
        xb = oracle.pubkey(i)[0].to_bytes(32, "big")
        u = int.from_bytes(xb[8:12], "big")
        s = [int.from_bytes(xb[12 + 4 * q:16 + 4 * q], "big") for q in range(2)]
        base = xb[0] * blocks * 16 + ((u * blocks) >> 32) * 16
        for w in range(4):
            a = s[w // 2] >> (8 * (w % 2))
            for v in (a, a >> 4):
                for f in (v & 15, 16 + ((v >> 16) & 15)):
                    model[base + 4 * w + (f >> 3)] |= 1 << (f & 7)
    assert engine.get_bloom(1) == bytes(model)


def test_candidate_overflow_grows_and_redoes_round(oracle, monkeypatch):
    """A round with more first-level candidates than the buffer holds is walked again with a
    larger buffer: same key, same candidate count as an unconstrained run."""
    from keyhunt_amd import Engine
    n, k = 1 << 40, 1                       # 2^20 giant points per base: a few candidates
    key = 0x3A5F0C3D2B1E00000 + 777
    out = []
    for cap in (None, "2"):
        if cap:
            monkeypatch.setenv("KH_CAND_CAP", cap)
        e = Engine(0)
        p = e.bsgs_setup(n, k, layer1=0)
        e.bsgs_build()
        e.bsgs_set_targets([oracle.pubkey(key)])
        start = key - 60 * 2 * p.n - 12345
        out.append((e.bsgs_scan(start, 64), e.bsgs_candidates()))
        e.close()
    assert out[0][0] == out[1][0] == [(0, key)]
    assert out[0][1] == out[1][1] > 2


def test_scan_list_equals_scan(engine, oracle):
    """kh_bsgs_scan_list over the same consecutive bases = kh_bsgs_scan (keys and candidates), and a
    shuffled, non-consecutive list finds the key in whichever base holds it."""
    import random
    n, k = 1 << 26, 4
    p = engine.bsgs_setup(n, k, layer1=0)
    engine.bsgs_build()
    key = 0x7CCE5EFDACCF6808
    engine.bsgs_set_targets([oracle.pubkey(key)])
    start = key - 5 * 2 * p.n - 4242
    c0 = engine.bsgs_candidates()
    a = engine.bsgs_scan(start, 8)
    c1 = engine.bsgs_candidates()
    engine.bsgs_reset_found()
    b = engine.bsgs_scan_list([start + i * 2 * p.n for i in range(8)])
    c2 = engine.bsgs_candidates()
    assert a == b == [(0, key)]
    assert c1 - c0 == c2 - c1
    engine.bsgs_reset_found()
    bases = [start + i * 2 * p.n for i in (11, 5, 2, 40, 7)]
    random.Random(3).shuffle(bases)
    assert engine.bsgs_scan_list(bases) == [(0, key)]
    engine.bsgs_reset_found()
    assert engine.bsgs_scan_list([start + 3 * 2 * p.n, start + 9 * 2 * p.n]) == []


@pytest.mark.parametrize("n,k", [(1 << 22, 2), (1 << 24, 3)])
def test_second_check_masks_gpu_equal_oracle(engine, oracle, n, k):
    """k_refine (the GPU second check) against the oracle's bsgs_secondcheck (keyhunt.cpp:5151-5184,
    AddDirect restated with its dx = 0 value) and the engine's host twin, bit for bit: base keys
    inside the target's 2M window (true layer-2 hits), random ones (FPs only), edges, and bases with
    S = +-AMP2[i] (the reference's AddDirect with dx = 0)."""
    import random
    rnd = random.Random(1234)
    p = oracle.bsgs_params(n, k)
    tabs = oracle.BsgsTables(p)
    engine.bsgs_setup(n, k)
    engine.bsgs_build()
    assert engine.get_bloom(2) == tabs.bf2.raw
    key = 0x3F00DEADBEEF0123
    engine.bsgs_set_targets([oracle.pubkey(key)])
    near = [key - rnd.randrange(0, 2 * p.m) for _ in range(600)]
    far = [rnd.getrandbits(255) for _ in range(400)]
    edge = [key, key - 2 * p.m, key - 2 * p.m + 1, 1, SECP_N - 1, 0]
    # S = Q - base*G = +-AMP2[i]: the reference's AddDirect with dx = 0 (inverse taken as 0)
    amp = [key + s * p.m2 * (1 + 2 * i) for i in (0, 5, 31) for s in (1, -1)]
    bases = near + far + edge + amp
    g, h = engine.bsgs_second_masks(0, bases)
    assert g == h
    assert g == oracle.bsgs_second_masks(tabs, bases, oracle.pubkey(key))
    hits = [m for m in g[: len(near)] if m]
    assert len(hits) >= 590   # d in [1, 2M): the AMP2 step covering d hits layer 2
    assert all(bin(m).count("1") <= 2 for m in hits)
    assert g[len(near) + len(far) + 5] == 0  # base key 0: no point
    assert len(g) == len(bases)


@pytest.mark.parametrize("mode", ["continuous", "per_base", "list"])
def test_gpu_refine_equals_host_refine(mode, oracle, monkeypatch):
    """Same found keys and the same first/second-level counts whether the second check runs in
    k_refine or on host threads (KH_REFINE=host), in the three scan modes."""
    import keyhunt_amd as K
    n, k = (1 << 22, 2) if mode != "per_base" else (1 << 24, 3)
    p = oracle.bsgs_params(n, k)
    keys = [0x1234567890ABCDE, 0x1234567890ABCDE + 7 * 2 * p.n + 99]
    start = keys[0] - 3 * 2 * p.n - 777
    res = []
    for how in ("gpu", "host"):
        if how == "host":
            monkeypatch.setenv("KH_REFINE", "host")
        else:
            monkeypatch.delenv("KH_REFINE", raising=False)
        with K.Engine(0) as e:
            e.bsgs_setup(n, k)
            e.bsgs_build()
            e.bsgs_set_targets([oracle.pubkey(x) for x in keys])
            if mode == "list":
                found = e.bsgs_scan_list([start + b * 2 * p.n for b in range(12)])
            else:
                found = e.bsgs_scan(start, 12)
            res.append((sorted(found), e.bsgs_refine_stats()))
    assert res[0] == res[1]
    assert sorted(res[0][0]) == [(0, keys[0]), (1, keys[1])]
    assert res[0][1][1] >= 2


@pytest.mark.parametrize("mode", ["per_base", "list"])
def test_device_centres_equal_host_centres(mode, oracle, monkeypatch):
    """Per-base rounds derive their lane scalars on the device (k_setup prog 2) or on the host
    (KH_HOST_CENTRES): same keys, same first-level candidates, same second-level hits; and a list
    reaching up to the group order (host path by the engine's own check) still finds its key."""
    import random
    import keyhunt_amd as K
    n, k = (1 << 22, 2) if mode == "list" else (1 << 24, 3)
    p = oracle.bsgs_params(n, k)
    keys = [0x2468ACE13579BDF, 0x2468ACE13579BDF + 9 * 2 * p.n + 4321]
    start = keys[0] - 4 * 2 * p.n - 999
    res = []
    for how in ("device", "host"):
        if how == "host":
            monkeypatch.setenv("KH_HOST_CENTRES", "1")
        else:
            monkeypatch.delenv("KH_HOST_CENTRES", raising=False)
        with K.Engine(0) as e:
            e.bsgs_setup(n, k)
            e.bsgs_build()
            e.bsgs_set_targets([oracle.pubkey(x) for x in keys])
            c0 = e.bsgs_candidates()
            if mode == "list":
                bases = [start + b * 2 * p.n for b in range(16)]
                random.Random(5).shuffle(bases)
                found = e.bsgs_scan_list(bases)
            else:
                found = e.bsgs_scan(start, 16)
            res.append((sorted(found), e.bsgs_candidates() - c0, e.bsgs_refine_stats()[1]))
    assert res[0] == res[1]
    assert res[0][0] == [(0, keys[0]), (1, keys[1])]
    monkeypatch.delenv("KH_HOST_CENTRES", raising=False)
    with K.Engine(0) as e:
        e.bsgs_setup(n, k)
        e.bsgs_build()
        key = SECP_N - 2 * p.n + 12345
        e.bsgs_set_targets([oracle.pubkey(key)])
        bases = [0x1111111111111111, key - 6000, SECP_N - 3 * p.n]
        assert e.bsgs_scan_list(bases) == [(0, key)]


def test_large_calls_use_wide_lanes_same_results(engine, oracle):
    """A call of >= 2^21 walk groups runs 2^21 lanes, >= 2^20 groups 2^20 lanes, smaller calls 2^18:
    one call over 2^19 bases, the same bases in two and in four calls, and as a shuffled list all
    probe the same points (same first-level candidates) and find the key in the same base."""
    import random
    # M = 2^22: 16384 entries per shard, past the 10000-entry floor, so layer 1 has false positives
    # to compare; 16384 giant points per base = 4 groups of 4096
    n, k = 1 << 36, 16
    p = oracle.bsgs_params(n, k)
    engine.bsgs_setup(n, k, layer1=1)
    engine.bsgs_build()
    nb = 1 << 19
    start = 0x5A5A5A5A5A0000000
    key = start + (nb - 3) * 2 * p.n + 31337
    far = start - 12345 * 2 * p.n       # no base of the call holds it: every point is walked
    bases = [start + b * 2 * p.n for b in range(nb)]
    random.Random(11).shuffle(bases)
    runs = []
    for tgt in (far, key):
        for plan in (1, 2, 4, "list"):
            engine.bsgs_set_targets([oracle.pubkey(tgt)])
            c0 = engine.bsgs_candidates()
            if plan == "list":
                got = engine.bsgs_scan_list(bases)
            else:
                got = []
                for i in range(plan):
                    got += engine.bsgs_scan(start + i * (nb // plan) * 2 * p.n, nb // plan)
            runs.append((tgt, plan, got, engine.bsgs_candidates() - c0))
    assert [r[2] for r in runs[:4]] == [[]] * 4
    assert len({r[3] for r in runs[:4]}) == 1 and runs[0][3] > 0
    assert [r[2] for r in runs[4:]] == [[(0, key)]] * 4


# Past the 10000-entry floor (keyhunt.cpp:7605-7626): n = 2^36, k = 16 gives M = 2^22, 16384 babies per
# shard, so layer 1 has false positives at its design rate (~6.6e-7 per giant point, ~0.011 per base of
# 16384 giant points = 4 groups of 4096).  The tests below walk thousands of bases, so "same first-level
# candidates" compares dozens of candidates, not zero with zero, and each also checks the giant points
# the walk counted (kh_kernel_time: n_bases x 16384 for a call that finds nothing), so a group skipped
# or walked twice fails even where no candidate falls in it.
N36, K16 = 1 << 36, 16


def _walked(e):
    from keyhunt_amd.engine import TIME_BSGS
    return e.kernel_time(TIME_BSGS)[2]


@pytest.mark.parametrize("lanes,calls", [(1024, [1501, 1501, 333]), (1024, [1536, 1536, 256]), (512, [900, 900, 900])])
def test_calls_with_ragged_lane_tiles(oracle, lanes, calls):
    """Calls whose groups the lanes do not tile exactly (1501 bases = 6004 groups over 1024 lanes: 6
    groups per lane on 1001 lanes, 2 unprobed lane-groups past the end) give the same candidates and keys
    as one call over all the bases: a following call starts its lanes again rather than continuing lanes
    that ended past its first group.  The other cases tile exactly (1024 x 6, 512 -> 450 x 8)."""
    import keyhunt_amd as K
    p = oracle.bsgs_params(N36, K16)
    assert p.aux == 16384
    total = sum(calls)
    start = 0x13579BDF02468000
    key = start + (calls[0] + calls[1] // 2) * 2 * p.n + 2024   # in the second call
    far = start - 99 * 2 * p.n
    with K.Engine(0, lanes, 0) as e:
        e.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
        e.bsgs_build()
        res = []
        for plan in ([total], calls):
            for tgt in (far, key):
                e.bsgs_set_targets([oracle.pubkey(tgt)])
                c0 = e.bsgs_candidates()
                e.kernel_time_reset()
                got, b = [], 0
                for nb in plan:
                    got += e.bsgs_scan(start + b * 2 * p.n, nb)
                    b += nb
                res.append((got, e.bsgs_candidates() - c0, _walked(e)))
    assert res[0][0] == res[2][0] == []
    assert res[0][1] == res[2][1] and res[0][1] > 0    # the same first-level false positives
    assert res[0][2] == res[2][2] == total * p.aux     # every giant point walked once
    assert res[1][0] == res[3][0] == [(0, key)]


@pytest.mark.parametrize("cands,stages", [(1, 1), (2, 2), (3, 2), ("move", 1)])
def test_placement_calibration_same_results(oracle, monkeypatch, cands, stages):
    """A context's first call of >= 2^23 walk groups walks its parts on candidate placements and keeps the
    fastest: by default 2^21 and 2^20 lanes on the one pad (A B B A); opt-in, several pads held at once
    (KH_PAD_CANDIDATES, A B C C B A) then a layer-1 copy (KH_CAL_STAGES=2), or the pad moved
    (KH_CAL_MOVE=1).  The same first-level candidates and walked points as an uncalibrated call
    (KH_BSGS_CALIBRATE=0), the key found in any part, and kh_bsgs_geometry / kh_bsgs_placement report the
    kept and the best other candidates' rates."""
    import keyhunt_amd as K
    p = oracle.bsgs_params(N36, K16)
    nb = 1 << 22                           # 4 groups per base: 8 x 2^21 groups, both stages in one call
    start = 0x3C3C3C3C3C000000
    far = start - 777 * 2 * p.n
    if cands == "move":
        monkeypatch.setenv("KH_CAL_MOVE", "1")
    else:
        monkeypatch.setenv("KH_PAD_CANDIDATES", str(cands))
    monkeypatch.setenv("KH_CAL_STAGES", str(stages))
    res = []
    for calibrate in (True, False):
        if calibrate:
            monkeypatch.delenv("KH_BSGS_CALIBRATE", raising=False)
        else:
            monkeypatch.setenv("KH_BSGS_CALIBRATE", "0")
        with K.Engine(0) as e:
            e.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
            e.bsgs_build()
            e.bsgs_set_targets([oracle.pubkey(far)])
            c0 = e.bsgs_candidates()
            assert e.bsgs_scan(start, nb) == []
            res.append((e.bsgs_candidates() - c0, _walked(e), e.bsgs_geometry(), e.bsgs_placement()))
    assert res[0][0] == res[1][0] and res[0][0] > 1000
    assert res[0][1] == res[1][1] == nb * p.aux
    lanes, r_kept, r_other = res[0][2]
    assert lanes in (1 << 21, 1 << 20) and r_kept > 0 and r_other > 0
    assert cands == "move" or r_kept >= r_other   # a move keeps its last placement whatever it measured
    done, rates = res[0][3]
    assert done and rates[0] == r_kept
    assert (rates[2] >= rates[3] > 0) if stages == 2 else rates[2:] == [0.0, 0.0]
    assert res[1][2] == (0, 0.0, 0.0) and res[1][3] == (False, [0.0] * 4)
    monkeypatch.delenv("KH_BSGS_CALIBRATE", raising=False)
    for where in (3, nb // 2 - 7, nb - 5):  # the key in the first, a middle and the last part
        key = start + where * 2 * p.n + 999
        with K.Engine(0) as e:
            e.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
            e.bsgs_build()
            e.bsgs_set_targets([oracle.pubkey(key)])
            assert e.bsgs_scan(start, nb) == [(0, key)]


def test_release_walk_between_calls(engine, oracle):
    """kh_release_walk frees the lane arrays and the pad: the next call allocates them again and
    starts its lanes afresh, with the same candidates, walked points and key as uninterrupted calls."""
    import keyhunt_amd as K
    p = oracle.bsgs_params(N36, K16)
    engine.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
    engine.bsgs_build()
    start = 0x2468ACE0000000
    far = start - 4321 * 2 * p.n
    key = start + 3000 * 2 * p.n + 4242    # in the second call
    res = []
    for tgt in (far, key):
        for release in (False, True):
            engine.bsgs_set_targets([oracle.pubkey(tgt)])
            c0 = engine.bsgs_candidates()
            engine.kernel_time_reset()
            got = engine.bsgs_scan(start, 2048)
            if release:
                engine.release_walk()
            got += engine.bsgs_scan(start + 2048 * 2 * p.n, 2048)
            res.append((got, engine.bsgs_candidates() - c0, _walked(engine)))
    assert res[0] == res[1] and res[0][0] == [] and res[0][1] > 0 and res[0][2] == 4096 * p.aux
    assert res[2][:2] == res[3][:2] and res[2][0] == [(0, key)]


def test_bsgs_lanes_continue_across_calls(engine, oracle):
    """Continuous mode keeps its (interleaved) lanes across kh_bsgs_scan calls whose bases follow
    on: scanning 4096 bases in one call, in 4 calls of 1024, in uneven calls, or with a jump and a
    target switch in between gives the same first-level candidates and walked points and finds the key
    in the same base."""
    import keyhunt_amd as K
    from keyhunt_amd.engine import TIME_SETUP
    p = oracle.bsgs_params(N36, K16)
    engine.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
    engine.bsgs_build()
    total = 4096
    start = 0x1234567890000
    key = start + 4000 * 2 * p.n + 777     # in the last call of every plan
    far = start + 1000000 * 2 * p.n   # past every base these calls walk
    for tgt in (far, key):
        q = oracle.pubkey(tgt)
        engine.bsgs_set_targets([q])
        c0 = engine.bsgs_candidates()
        engine.kernel_time_reset()
        one = engine.bsgs_scan(start, total)
        one_call = (engine.bsgs_candidates() - c0, _walked(engine))
        assert one == ([] if tgt == far else [(0, key)])
        assert one_call[0] > 0 and one_call[1] == total * p.aux
        for plan in ([1024] * 4, [512, 512, 1536, 1536], "jump"):
            engine.bsgs_set_targets([q])
            c0 = engine.bsgs_candidates()
            got, b = [], 0
            if plan == "jump":                 # an unrelated range, a second target, then back
                engine.bsgs_scan(start + 100000 * 2 * p.n, 64)
                engine.bsgs_set_targets([oracle.pubkey(tgt + 5)])
                engine.bsgs_scan(start, 64)
                engine.bsgs_set_targets([q])
                c0 = engine.bsgs_candidates()
                plan = [1536, 2560]
            engine.kernel_time_reset()
            for nb in plan:
                got += [(b, f) for f in engine.bsgs_scan(start + b * 2 * p.n, nb)]
                b += nb
            if tgt == key:
                assert [f for _, f in got] == [(0, key)]
                assert got[0][0] + plan[-1] == total
            else:
                assert got == []
            if plan == [1024] * 4:             # the lanes were started once, then continued
                assert engine.kernel_time(TIME_SETUP)[0] == 1
            assert (engine.bsgs_candidates() - c0, _walked(engine)) == one_call, plan


def test_pad_skew_and_offset_same_results(oracle, monkeypatch):
    """The pad layout knobs (KH_PAD_SKEW: a gap of lanes after every pad row, honoured by the kernels of
    a -DKH_PAD_KNOBS=1 build; KH_PAD_OFFSET: the pad's start inside its allocation) move only where the
    inversion pad sits: the same first-level candidates, walked points and key as the default layout, for
    the BSGS walk and an xpoint chunk."""
    import keyhunt_amd as K
    p = oracle.bsgs_params(N36, K16)
    start = 0x7777777700000
    key = start + 3000 * 2 * p.n + 31
    xkeys = [(1 << 61) + 12345 + 99991 * j for j in range(5)]
    xrows = [oracle.pubkey(k)[0].to_bytes(32, "big")[:20] for k in xkeys]
    res = []
    for skew, off in ((None, None), ("37", "4096"), ("3000", "65792")):
        for var, val in (("KH_PAD_SKEW", skew), ("KH_PAD_OFFSET", off)):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        with K.Engine(0) as e:
            e.bsgs_setup(N36, K16, layer1=K.KH_LAYER1_BLOCKED)
            e.bsgs_build()
            e.bsgs_set_targets([oracle.pubkey(key)])
            got = e.bsgs_scan(start, 4096)
            walked = _walked(e)
            e.set_targets(xrows)
            xs = sorted(h.key for h in e.scan(1 << 61, 1 << 24, mode=K.KH_MODE_XPOINT, search=0))
            res.append((got, e.bsgs_candidates(), walked, xs))
    assert res[0][0] == [(0, key)] and res[0][1] > 0 and res[0][3] == sorted(xkeys)
    assert res[1] == res[0] and res[2] == res[0]
