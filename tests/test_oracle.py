"""The CPU oracle (oracle/kh_oracle.c) pinned against the reference: primitive vectors printed by the
reference's own code (tests/golden/ref_vectors.json) and the reference CLI's hit sets on
known-answer windows (tests/golden/ref_e2e.json)."""
import hashlib
import json
import os
import random

import pytest

from conftest import GOLDEN

VEC = json.load(open(os.path.join(GOLDEN, "ref_vectors.json")))
E2E = json.load(open(os.path.join(GOLDEN, "ref_e2e.json")))
P = 2**256 - 2**32 - 977


def h(x):
    return int(x, 16)


def test_field_vs_reference(oracle):
    for v in VEC["field"]:
        a, b = h(v["a"]), h(v["b"])
        assert oracle.fe_mul(a, b) == h(v["mul"]) % P
        assert oracle.fe_mul(a, a) == h(v["sqr"]) % P
        assert oracle.fe_inv(a) == h(v["inv"])


def test_pubkeys_and_hash160_vs_reference(oracle):
    for v in VEC["pubkeys"]:
        x, y = oracle.pubkey(h(v["k"]))
        assert (x, y) == (h(v["x"]), h(v["y"]))
        assert oracle.hash160_comp(x, 2).hex() == v["h02"]
        assert oracle.hash160_comp(x, 3).hex() == v["h03"]
        assert oracle.hash160_uncomp(x, y).hex() == v["h04"]
        assert oracle.decompress(x, y & 1) == y


def test_xxh64_vs_reference(oracle):
    for v in VEC["xxh64"]:
        buf = bytes.fromhex(v["buf"])
        a = oracle.xxh64(buf, 0x59F2815B16F81798)
        assert a == h(v["a"])
        assert oracle.xxh64(buf, a) == h(v["b"])


def test_bloom_sizing_vs_reference(oracle):
    for v in VEC["bloom_params"]:
        assert oracle.bloom_params(v["entries"]) == (v["bits"], v["bytes"], v["hashes"])


def test_bloom_fill_vs_reference(oracle):
    fill = VEC["bloom_fill"]
    b = oracle.Bloom(fill["entries"])
    items = [bytes.fromhex(x) for x in fill["items"]]
    for it in items:
        b.add(it)
    assert hashlib.sha256(b.raw()).hexdigest() == fill["sha256"]
    assert all(b.check(it) for it in items)


def test_group_walk_vs_reference(oracle):
    for gw in VEC["group_walk"]:
        xs, _ = oracle.walk_points(h(gw["start"]), gw["n"] // 1024)
        assert hashlib.sha256(xs).hexdigest() == gw["sha256_walk"] == gw["sha256_direct"]


@pytest.mark.parametrize("cfg", VEC["bsgs_build"][:2], ids=lambda c: f"n{c['n']:x}_k{c['k']}")
def test_bsgs_build_vs_reference(oracle, cfg):
    p = oracle.bsgs_params(cfg["n"], cfg["k"])
    assert (p.m, p.m2, p.m3) == (cfg["m"], cfg["m2"], cfg["m3"])
    t = oracle.BsgsTables(p)
    assert hashlib.sha256(t.bf1.raw).hexdigest() == cfg["sha256_l1"]
    assert hashlib.sha256(t.bf2.raw).hexdigest() == cfg["sha256_l2"]
    assert hashlib.sha256(t.bf3.raw).hexdigest() == cfg["sha256_l3"]
    assert hashlib.sha256(t.table_bytes()).hexdigest() == cfg["sha256_table"]


def test_bsgs_params_configs(oracle):
    """BASELINE configs 4/5 geometry."""
    p = oracle.bsgs_params(2**44, 128)
    assert (p.m, p.m2, p.m3, p.cycles) == (2**29, 2**24, 2**19, 32)
    assert (p.bits[0], p.bytes[0], p.hashes[0]) == (60303973, 7537997, 20)
    assert (p.bytes[1], p.bytes[2]) == (235563, 35944)
    p = oracle.bsgs_params(2**44, 512)
    assert (p.m, p.m2, p.m3, p.cycles) == (2**31, 2**26, 2**21, 8)
    assert (p.bytes[0], p.bytes[1]) == (30151987, 942250)


def _read_rows(oracle, fn, mode):
    from conftest import DATA
    rows = []
    for line in open(os.path.join(DATA, fn)):
        s = line.strip()
        if mode == "xpoint":
            if len(s) in (64, 66):
                rows.append(bytes.fromhex(s[-64:])[:20])
            continue
        if len(s) == 40:
            rows.append(bytes.fromhex(s))
        elif 20 < len(s) < 40:
            raw = oracle.address_decode(s)
            if raw:
                rows.append(raw[1:21])
    return rows


@pytest.mark.parametrize("name,fn,mode,search,endo", [
    ("rmd160_1to32_compress_2p20", "1to32.rmd", 0, 0, False),
    ("xpoint_1to63_65_2p20", "1to63_65.txt", 1, 2, False),
    ("rmd160_1to32_compress_2p20_endo", "1to32.rmd", 0, 0, True),
    ("xpoint_1to63_65_2p20_endo", "1to63_65.txt", 1, 2, True),
    ("address_endo_targets", "endo_addr.txt", 0, 2, True),
    ("address_endo_targets_no_e", "endo_addr.txt", 0, 2, False),
    ("xpoint_endo_targets", "endo_x.txt", 1, 2, True),
])
def test_oracle_scan_vs_reference_cli(oracle, name, fn, mode, search, endo):
    """Keys 1..2^20 (one 2^20 chunk): the oracle's hit list equals the reference CLI's, with and
    without -e (endo_*.txt hold lambda-multiples of small keys, tests/golden/make_endo_targets.py)."""
    rows = _read_rows(oracle, fn, "xpoint" if mode == 1 else "addr")
    hits = oracle.scan_chunk(mode, search, 1, 1 << 20, rows, endo=endo)
    assert [f"{k:x}" for k in sorted(k for k, _, _ in hits)] == [x["key"] for x in E2E[name]["hits"]]


@pytest.mark.parametrize("name,search,endo,group", [
    ("rmd160_batch512_compress", 0, False, 512),
    ("rmd160_batch512_both", 2, False, 512),
    ("rmd160_batch512_both_endo", 2, True, 512),
    ("rmd160_batch1000_compress", 0, False, 1000),
    ("rmd160_batch1000_both", 2, False, 1000),
    ("rmd160_batch1001_compress_endo", 0, True, 1000),  # the reference rounds 1001 down to 1000
    ("rmd160_batch1024_both", 2, False, 1024),
])
def test_oracle_rmd_batch_vs_reference_cli(oracle, name, search, endo, group):
    """-m rmd160 --rmd-batch-size G over 0x10000..0x20ffff in two 2^20 chunks: the oracle's walk
    (the reference's partly zero batch inversion restated, kh_oracle.c walk_group_n) finds exactly
    the reference CLI's keys -- group centres, and the negated or nominal slot keys of the points
    that are no multiples of G (tests/golden/make_rmd_batch_targets.py)."""
    assert E2E[name]["argv"][E2E[name]["argv"].index("--rmd-batch-size") + 1] in (str(group), str(group + 1))
    rows = _read_rows(oracle, "rmd_batch.rmd", "addr")
    keys = []
    for chunk in range(2):
        keys += [k for k, _, _ in oracle.scan_chunk(0, search, 0x10000 + chunk * (1 << 20), 1 << 20, rows,
                                                    endo=endo, group=group)]
    assert [f"{k:x}" for k in sorted(keys)] == [x["key"] for x in E2E[name]["hits"]]


def test_oracle_scan_window_66(oracle):
    rows = _read_rows(oracle, "66.rmd", "addr")
    start = 0x2832ED74F2B5E0000
    hits = oracle.scan_chunk(0, 0, start, 1 << 16, rows)
    assert [(f"{k:x}", c) for k, c, _ in hits] == [("2832ed74f2b5e35ee", True)]
    assert [x["key"] for x in E2E["rmd160_66_window"]["hits"]] == ["2832ed74f2b5e35ee"]


def test_oracle_bsgs_known_answer_small_n(oracle):
    """-m bsgs -f 63.pub -n 0x1000000 -k 4 -r 7cce5efdac000000:7cce5efdad000000 (reference: found)."""
    p = oracle.bsgs_params(1 << 24, 4)
    t = oracle.BsgsTables(p)
    q = oracle.parse_pubkey_hex(open(os.path.join(GOLDEN, "data", "63.pub")).read().split()[0])
    key, cands = t.scan(0x7CCE5EFDAC000000, 1, q)
    assert f"{key:x}" == E2E["bsgs_63_small_n_k4"]["hits"][0]["key"]
    assert len(cands) >= 1


def test_searchbinary_is_membership(oracle):
    """keyhunt's midpoint loop (keyhunt.cpp:3065-3089) answers exact membership on sorted tables."""
    rng = random.Random(3)
    for n in list(range(1, 40)) + [100, 1000, 4097]:
        rows = sorted({rng.getrandbits(160).to_bytes(20, "big") for _ in range(n)})
        table = b"".join(rows)
        for r in rows:
            assert oracle.searchbinary(table, len(rows), r)
        for _ in range(50):
            q = rng.getrandbits(160).to_bytes(20, "big")
            assert oracle.searchbinary(table, len(rows), q) == (q in set(rows))


def test_oracle_keccak_and_eth_against_reference_vectors(oracle):
    """The oracle's Keccak-256 / generate_binaddress_eth against the reference's (ref_golden "eth")."""
    for v in VEC["eth"]:
        x, y = oracle.pubkey(int(v["k"], 16))
        assert (x.to_bytes(32, "big") + y.to_bytes(32, "big")).hex() == v["xy"]
        assert oracle.keccak256(bytes.fromhex(v["xy"])).hex() == v["keccak"]
        assert oracle.eth_address(x, y).hex() == v["address"]


def test_oracle_second_masks_window(oracle):
    """bsgs_secondcheck's layer-2 probes (keyhunt.cpp:5151-5184): for base = key - d, S = d*G and
    S + AMP2[i] = (d - (2i+1)M2)*G, whose X is a layer-2 baby X exactly when |d - (2i+1)M2| is in
    [1, M2]: bit min(d // (2 M2), 31) is set for every d in [1, 64 M2] but the odd multiples of M2
    (there S = -AMP2[i], AddDirect's dx = 0); other bits only as FPs.  Base key 0 gives 0."""
    import random
    p = oracle.bsgs_params(1 << 22, 2)
    t = oracle.BsgsTables(p)
    key = 0x3F00DEADBEEF0123
    q = oracle.pubkey(key)
    rnd = random.Random(7)
    ds = [1, p.m2 - 1, p.m2 + 1, 2 * p.m2, 64 * p.m2] + [rnd.randrange(1, 64 * p.m2 + 1) for _ in range(60)]
    ds = [d for d in ds if d % (2 * p.m2) != p.m2]
    masks = oracle.bsgs_second_masks(t, [key - d for d in ds], q)
    for d, m in zip(ds, masks):
        assert (m >> min(d // (2 * p.m2), 31)) & 1, (d, hex(m))
    assert oracle.bsgs_second_masks(t, [0], q) == [0]


def test_oracle_blocked_layer1_check_vs_spec_model(oracle):
    """or_blk_check (the oracle's probe of the engine's blocked layer 1) against a filter written
    from the layout's specification in Python (the same model test_blocked_layer1_bytes_match_
    layout_spec pins the GPU build to): every inserted X passes, and random X's pass at about the
    fill-implied rate only."""
    import ctypes
    rng = random.Random(5)
    blocks = 64
    model = bytearray(256 * blocks * 16)

    def words(xb):
        base = xb[0] * blocks * 16 + ((int.from_bytes(xb[8:12], "big") * blocks) >> 32) * 16
        s = [int.from_bytes(xb[12 + 4 * q:16 + 4 * q], "big") for q in range(2)]
        for w in range(4):
            a = s[w // 2] >> (8 * (w % 2))
            for v in (a, a >> 4):
                for f in (v & 15, 16 + ((v >> 16) & 15)):
                    yield base + 4 * w + (f >> 3), 1 << (f & 7)

    ins = [rng.getrandbits(256).to_bytes(32, "big") for _ in range(3000)]
    for xb in ins:
        for off, bit in words(xb):
            model[off] |= bit
    buf = ctypes.create_string_buffer(bytes(model), len(model))
    chk = oracle.lib().or_blk_check
    assert all(chk(buf, ctypes.c_uint64(blocks), xb) == 1 for xb in ins)
    rnd = [rng.getrandbits(256).to_bytes(32, "big") for _ in range(20000)]
    hits = sum(chk(buf, ctypes.c_uint64(blocks), xb) for xb in rnd)
    # a random X passes iff all 16 of its bits are set: the model says so too
    exp = sum(all(model[o] & b for o, b in words(xb)) for xb in rnd)
    assert hits == exp and hits < 200
