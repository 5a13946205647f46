"""ctypes wrapper around oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of keyhunt's hot path (see kh_oracle.c for the reference file:line each
function follows).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product (keyhunt_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None
SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_u8p = ctypes.c_char_p
        L.or_xxh64.restype = ctypes.c_uint64
        L.or_xxh64.argtypes = [c_u8p, ctypes.c_uint64, ctypes.c_uint64]
        L.or_bloom_params.argtypes = [ctypes.c_uint64, ctypes.c_double, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]
        L.or_bloom_entries.restype = ctypes.c_uint64
        L.or_bloom_entries.argtypes = [ctypes.c_uint64]
        L.or_bsgs_giant_probe.restype = ctypes.c_uint64
        _lib = L
    return _lib


# ---------------------------------------------------------------------------------------------
# primitives
# ---------------------------------------------------------------------------------------------
def be32(v: int) -> bytes:
    return int(v).to_bytes(32, "big")


def sha256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_sha256(msg, ctypes.c_uint64(len(msg)), out)
    return out.raw


def ripemd160(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(20)
    lib().or_ripemd160(msg, ctypes.c_uint64(len(msg)), out)
    return out.raw


def xxh64(buf: bytes, seed: int) -> int:
    return lib().or_xxh64(buf, len(buf), ctypes.c_uint64(seed))


def fe_mul(a: int, b: int) -> int:
    out = ctypes.create_string_buffer(32)
    lib().or_fe_mul(be32(a), be32(b), out)
    return int.from_bytes(out.raw, "big")


def fe_inv(a: int) -> int:
    out = ctypes.create_string_buffer(32)
    lib().or_fe_inv(be32(a), out)
    return int.from_bytes(out.raw, "big")


def pubkey(k: int) -> tuple[int, int]:
    x = ctypes.create_string_buffer(32)
    y = ctypes.create_string_buffer(32)
    lib().or_pubkey(be32(k), x, y)
    return int.from_bytes(x.raw, "big"), int.from_bytes(y.raw, "big")


def decompress(x: int, odd: int) -> int:
    y = ctypes.create_string_buffer(32)
    ok = lib().or_decompress(be32(x), ctypes.c_int(odd), y)
    if not ok:
        raise ValueError("x not on curve")
    return int.from_bytes(y.raw, "big")


def point_add(a: tuple[int, int], b: tuple[int, int]) -> tuple[int, int]:
    rx = ctypes.create_string_buffer(32)
    ry = ctypes.create_string_buffer(32)
    lib().or_point_add(be32(a[0]), be32(a[1]), be32(b[0]), be32(b[1]), rx, ry)
    return int.from_bytes(rx.raw, "big"), int.from_bytes(ry.raw, "big")


def hash160_comp(x: int, prefix: int) -> bytes:
    out = ctypes.create_string_buffer(20)
    lib().or_hash160_comp(be32(x), ctypes.c_uint8(prefix), out)
    return out.raw


def hash160_uncomp(x: int, y: int) -> bytes:
    out = ctypes.create_string_buffer(20)
    lib().or_hash160_uncomp(be32(x), be32(y), out)
    return out.raw


def keccak256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_keccak256(msg, ctypes.c_uint64(len(msg)), out)
    return out.raw


def eth_address(x: int, y: int) -> bytes:
    """generate_binaddress_eth (keyhunt.cpp:5663-5669): Keccak-256(X||Y)[12:32]."""
    out = ctypes.create_string_buffer(20)
    lib().or_eth_address(be32(x), be32(y), out)
    return out.raw


def h160_to_address(h: bytes) -> str:
    out = ctypes.create_string_buffer(64)
    lib().or_h160_to_address(h, out, 64)
    return out.value.decode()


def address_decode(s: str) -> bytes | None:
    out = ctypes.create_string_buffer(25)
    r = lib().or_address_decode(s.encode(), out)
    return out.raw if r == 25 else None


# ---------------------------------------------------------------------------------------------
# bloom
# ---------------------------------------------------------------------------------------------
def bloom_params(entries: int, error: float = 1e-6) -> tuple[int, int, int]:
    bits = ctypes.c_uint64()
    nbytes = ctypes.c_uint64()
    hashes = ctypes.c_uint32()
    r = lib().or_bloom_params(entries, error, ctypes.byref(bits), ctypes.byref(nbytes), ctypes.byref(hashes))
    if r:
        raise ValueError("bad bloom params")
    return bits.value, nbytes.value, hashes.value


def bloom_entries(items: int) -> int:
    return lib().or_bloom_entries(items)


def bloom_positions(bits: int, hashes: int, buf: bytes) -> list[int]:
    out = (ctypes.c_uint64 * hashes)()
    lib().or_bloom_positions(ctypes.c_uint64(bits), ctypes.c_uint32(hashes), buf, ctypes.c_int(len(buf)), out)
    return list(out)


class Bloom:
    """Reference-layout bloom filter (bloom/bloom.cpp)."""

    def __init__(self, items: int):
        self.bits, self.nbytes, self.hashes = bloom_params(bloom_entries(items))
        self.bf = ctypes.create_string_buffer(self.nbytes)

    def add(self, buf: bytes) -> None:
        lib().or_bloom_add(self.bf, ctypes.c_uint64(self.bits), ctypes.c_uint32(self.hashes), buf, len(buf))

    def check(self, buf: bytes) -> bool:
        return bool(lib().or_bloom_check(self.bf, ctypes.c_uint64(self.bits), ctypes.c_uint32(self.hashes), buf, len(buf)))

    def raw(self) -> bytes:
        return self.bf.raw


def searchbinary(rows: bytes, n: int, key: bytes, width: int = 20, key_off: int = 0) -> bool:
    return bool(lib().or_searchbinary(rows, ctypes.c_int64(n), key, ctypes.c_int(width), ctypes.c_int(key_off)))


# ---------------------------------------------------------------------------------------------
# group walk / scan
# ---------------------------------------------------------------------------------------------
def walk_points(start: int, n_groups: int, stride: int = 1, need_y: bool = False):
    n = n_groups * 1024
    xs = ctypes.create_string_buffer(32 * n)
    ys = ctypes.create_string_buffer(32 * n) if need_y else None
    lib().or_walk_points(be32(start), be32(stride), ctypes.c_uint64(n_groups), xs, ys)
    return xs.raw, (ys.raw if need_y else None)


class OrHit(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint8 * 32), ("compressed", ctypes.c_int32), ("kind", ctypes.c_int32)]


MODE_ADDRESS = 0   # address / rmd160 share the hash160 probe
MODE_XPOINT = 1
MODE_ETH = 2       # -c eth: Keccak-256(X||Y)[12:32] probes
SEARCH_COMPRESS, SEARCH_UNCOMPRESS, SEARCH_BOTH = 0, 1, 2


def scan_chunk(mode: int, search: int, start: int, n_keys: int, rows: list[bytes], cap: int = 4096,
               endo: bool = False, group: int = 1024):
    """Reference hit list for one chunk (thread_process).  rows: 20-byte targets (unsorted ok).
    endo: -e (kinds then carry the image e << 4 and, for 04 hashes, the Y sign << 6).  group:
    -m rmd160 --rmd-batch-size after the reference's clamping (kh_oracle.c walk_group_n)."""
    srt = sorted(rows)
    table = b"".join(srt)
    bloom = Bloom(len(srt))
    for r in srt:
        bloom.add(r)
    hits = (OrHit * cap)()
    n = lib().or_scan_chunk3(ctypes.c_int(mode), ctypes.c_int(search), ctypes.c_int(1 if endo else 0),
                             ctypes.c_int(group), be32(start),
                             ctypes.c_uint64(n_keys),
                            table, ctypes.c_int64(len(srt)), bloom.bf, ctypes.c_uint64(bloom.bits),
                            ctypes.c_uint32(bloom.hashes), hits, ctypes.c_int(cap))
    return [(int.from_bytes(bytes(h.key), "big"), bool(h.compressed), int(h.kind)) for h in hits[: min(n, cap)]]


# ---------------------------------------------------------------------------------------------
# BSGS
# ---------------------------------------------------------------------------------------------
class BsgsParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("m", ctypes.c_uint64), ("m2", ctypes.c_uint64), ("m3", ctypes.c_uint64),
                ("aux", ctypes.c_uint64), ("cycles", ctypes.c_uint64), ("items1", ctypes.c_uint64),
                ("items2", ctypes.c_uint64), ("items3", ctypes.c_uint64), ("bits", ctypes.c_uint64 * 3),
                ("bytes", ctypes.c_uint64 * 3), ("hashes", ctypes.c_uint32 * 3)]


class BxRow(ctypes.Structure):
    _fields_ = [("value", ctypes.c_uint8 * 6), ("pad", ctypes.c_uint8 * 2), ("index", ctypes.c_uint64)]


def bsgs_params(n: int, k: int) -> BsgsParams:
    p = BsgsParams()
    r = lib().or_bsgs_params_compute(ctypes.c_uint64(n), ctypes.c_uint64(k), ctypes.byref(p))
    if r:
        raise ValueError(f"invalid BSGS n/k ({r})")
    return p


class BsgsTables:
    def __init__(self, p: BsgsParams, build: bool = True):
        self.p = p
        self.l1_blocks = 0   # reference-layout layer 1
        self.bf1 = ctypes.create_string_buffer(256 * p.bytes[0])
        self.bf2 = ctypes.create_string_buffer(256 * p.bytes[1])
        self.bf3 = ctypes.create_string_buffer(256 * p.bytes[2])
        self.table = (BxRow * p.m3)()
        if build:
            lib().or_bsgs_build(ctypes.byref(p), self.bf1, self.bf2, self.bf3, self.table)

    @classmethod
    def from_raw(cls, p: BsgsParams, bf1: bytes, bf2: bytes, bf3: bytes, table: bytes,
                 l1_blocks: int = 0) -> "BsgsTables":
        """Tables given as bytes (reference layout), e.g. ones already checked byte-identical to the
        reference's: skips the oracle's own (slow, single-threaded) baby-step build.  l1_blocks != 0:
        bf1 is the engine's blocked layer 1 with that many 16-byte blocks per shard (or_blk_check)."""
        t = cls(p, build=False)
        t.l1_blocks = l1_blocks
        if l1_blocks:
            t.bf1 = ctypes.create_string_buffer(256 * 16 * l1_blocks)
        assert len(bf1) == len(t.bf1.raw) and len(bf2) == len(t.bf2.raw) and len(bf3) == len(t.bf3.raw)
        assert len(table) == ctypes.sizeof(t.table)
        ctypes.memmove(t.bf1, bf1, len(bf1))
        ctypes.memmove(t.bf2, bf2, len(bf2))
        ctypes.memmove(t.bf3, bf3, len(bf3))
        ctypes.memmove(t.table, table, len(table))
        return t

    def table_bytes(self) -> bytes:
        return ctypes.string_at(self.table, ctypes.sizeof(self.table))

    def scan(self, start: int, n_bases: int, q: tuple[int, int], cand_cap: int = 1 << 16):
        key = ctypes.create_string_buffer(32)
        cands = (ctypes.c_uint64 * (2 * cand_cap))()
        ncand = ctypes.c_uint64()
        found = lib().or_bsgs_scan_l1(ctypes.byref(self.p), self.bf1, ctypes.c_uint64(self.l1_blocks),
                                      self.bf2, self.bf3, self.table, be32(start),
                                      ctypes.c_uint64(n_bases), be32(q[0]), be32(q[1]), key, cands,
                                      ctypes.c_uint64(cand_cap), ctypes.byref(ncand))
        nc = min(ncand.value, cand_cap)
        cl = [(cands[2 * i], cands[2 * i + 1]) for i in range(nc)]
        return (int.from_bytes(key.raw, "big") if found else None), cl

    def refine(self, base: int, a: int, q: tuple[int, int]):
        key = ctypes.create_string_buffer(32)
        ok = lib().or_bsgs_refine(ctypes.byref(self.p), self.bf2, self.bf3, self.table, be32(base),
                                  ctypes.c_uint32(a), be32(q[0]), be32(q[1]), key)
        return int.from_bytes(key.raw, "big") if ok else None


def bsgs_second_masks(tabs: "BsgsTables", base_keys: list[int], q: tuple[int, int]) -> list[int]:
    """Layer-2 masks of bsgs_secondcheck (keyhunt.cpp:5151-5184) for the given base keys."""
    n = len(base_keys)
    buf = b"".join(be32(k % SECP_N) for k in base_keys) or bytes(32)
    out = (ctypes.c_uint32 * max(n, 1))()
    lib().or_bsgs_second_masks(ctypes.byref(tabs.p), tabs.bf2, buf, ctypes.c_uint64(n), be32(q[0]), be32(q[1]), out)
    return list(out[:n])


def bsgs_giant_probe(p: BsgsParams, bf1, q: tuple[int, int], n_groups_per_thread: int, threads: int) -> int:
    return lib().or_bsgs_giant_probe(ctypes.byref(p), bf1, be32(q[0]), be32(q[1]),
                                     ctypes.c_uint64(n_groups_per_thread), ctypes.c_int(threads))


def parse_pubkey_hex(s: str) -> tuple[int, int]:
    s = s.strip()
    if len(s) == 66:
        x = int(s[2:], 16)
        return x, decompress(x, int(s[:2], 16) & 1)
    if len(s) == 130:
        return int(s[2:66], 16), int(s[66:], 16)
    raise ValueError("bad pubkey hex")
