"""ctypes binding of include/kh_gpu.h (lib/libkh_gpu.so) -- the MI355X engine.

`Engine` mirrors the reference's worker seams (see include/kh_gpu.h for the keyhunt.cpp lines each
call replaces).  There is no CPU path here: if the shared library or the GPU is missing, calls
raise.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
from dataclasses import dataclass

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.environ.get("KH_LIB") or os.path.join(PKG, "lib", "libkh_gpu.so")
HEADER = os.path.join(REPO, "include", "kh_gpu.h")

KH_MODE_ADDRESS, KH_MODE_XPOINT, KH_MODE_ETH = 0, 1, 2
KH_MODE_ENDO = 0x10  # OR into mode: -e
KH_SEARCH_COMPRESS, KH_SEARCH_UNCOMPRESS, KH_SEARCH_BOTH = 0, 1, 2
KH_KIND_02, KH_KIND_03, KH_KIND_04, KH_KIND_XPOINT, KH_KIND_ETH = 0, 1, 2, 3, 5
KH_KIND_ENDO1, KH_KIND_ENDO2, KH_KIND_NEGY = 0x10, 0x20, 0x40
TIME_ADDRESS, TIME_XPOINT, TIME_BSGS, TIME_BUILD, TIME_SETUP = 0, 1, 2, 3, 4
KH_LAYER1_REFERENCE, KH_LAYER1_BLOCKED = 0, 1

ORDER_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


class KhError(RuntimeError):
    pass


class KhHit(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint8 * 32), ("offset", ctypes.c_uint64), ("kind", ctypes.c_uint32),
                ("compressed", ctypes.c_uint32)]


class KhBsgsInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("m", ctypes.c_uint64), ("m2", ctypes.c_uint64), ("m3", ctypes.c_uint64),
                ("aux", ctypes.c_uint64), ("cycles", ctypes.c_uint64), ("bloom_bits", ctypes.c_uint64 * 3),
                ("bloom_bytes", ctypes.c_uint64 * 3), ("bloom_hashes", ctypes.c_uint32 * 3),
                ("layer1_layout", ctypes.c_uint32)]


class KhBsgsFound(ctypes.Structure):
    _fields_ = [("target", ctypes.c_uint32), ("pad", ctypes.c_uint32), ("key", ctypes.c_uint8 * 32)]


_lib = None


def build(jobs: int = 8) -> str:
    subprocess.run(["make", "-s", "-C", PKG, f"-j{jobs}"], check=True)
    return LIB_PATH


def header_symbols() -> list[str]:
    """Every function the C-ABI header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(kh_\w+)\s*\(", txt, re.M)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KhError(f"{LIB_PATH} is missing: build the HIP engine first (python -c 'import keyhunt_amd; keyhunt_amd.build()')")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    u8p = ctypes.c_char_p
    L.kh_strerror.restype = ctypes.c_char_p
    L.kh_last_error.restype = ctypes.c_char_p
    L.kh_last_error.argtypes = [P]
    L.kh_open.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
    L.kh_close.argtypes = [P]
    L.kh_set_geometry.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32]
    L.kh_release_walk.argtypes = [P]
    L.kh_debug_layout.argtypes = [P, ctypes.POINTER(ctypes.c_uint64 * 8)]
    L.kh_bsgs_placement.argtypes = [P, ctypes.POINTER(ctypes.c_double * 4)]
    L.kh_debug_replace.argtypes = [P, ctypes.c_uint32]
    L.kh_debug_burn.argtypes = [P, ctypes.c_double]
    L.kh_bsgs_geometry.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_double * 2)]
    L.kh_synchronize.argtypes = [P]
    L.kh_scan_memory.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    L.kh_bsgs_set_bloom_multiplier.argtypes = [P, ctypes.c_uint32]
    L.kh_set_rmd_batch.argtypes = [P, ctypes.c_uint32]
    L.kh_set_targets.argtypes = [P, u8p, ctypes.c_uint64, ctypes.c_uint64]
    L.kh_set_vanity.argtypes = [P, u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
    L.kh_scan.argtypes = [P, u8p, u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(KhHit),
                          ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.kh_bsgs_setup.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(KhBsgsInfo)]
    L.kh_bsgs_set_layer1.argtypes = [P, ctypes.c_uint32]
    L.kh_bsgs_build.argtypes = [P]
    L.kh_bsgs_save.argtypes = [P, ctypes.c_char_p]
    L.kh_bsgs_load.argtypes = [P, ctypes.c_char_p, ctypes.c_uint32]
    L.kh_targets_save.argtypes = [P, ctypes.c_char_p]
    L.kh_targets_load.argtypes = [P, ctypes.c_char_p, ctypes.c_uint32]
    L.kh_bsgs_set_targets.argtypes = [P, u8p, ctypes.c_uint32]
    L.kh_bsgs_scan.argtypes = [P, u8p, ctypes.c_uint64, ctypes.POINTER(KhBsgsFound), ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32)]
    L.kh_bsgs_scan_list.argtypes = [P, u8p, ctypes.c_uint64, ctypes.POINTER(KhBsgsFound), ctypes.c_uint32,
                                    ctypes.POINTER(ctypes.c_uint32)]
    L.kh_bsgs_reset_found.argtypes = [P]
    L.kh_bsgs_candidates.argtypes = [P, ctypes.POINTER(ctypes.c_uint64)]
    L.kh_bsgs_refine_stats.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.kh_bsgs_second_masks.argtypes = [P, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint32)]
    L.kh_kernel_time.argtypes = [P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_uint64)]
    L.kh_kernel_time_reset.argtypes = [P]
    L.kh_pubkeys.argtypes = [P, u8p, ctypes.c_uint32, u8p]
    L.kh_walk_points.argtypes = [P, u8p, u8p, ctypes.c_uint64, u8p, u8p]
    L.kh_hash160.argtypes = [P, u8p, ctypes.c_uint32, u8p]
    L.kh_field_ops.argtypes = [P, u8p, u8p, ctypes.c_uint32, u8p]
    L.kh_bloom_check.argtypes = [P, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.c_uint32, u8p]
    L.kh_get_bloom.argtypes = [P, ctypes.c_uint32, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.kh_get_bsgs_table.argtypes = [P, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.kh_bsgs_set_table.argtypes = [P, u8p, ctypes.c_uint64]
    _lib = L
    return L


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().kh_device_count(ctypes.byref(n))
    return n.value


def be32(v: int) -> bytes:
    return (int(v) % (1 << 256)).to_bytes(32, "big")


@dataclass
class ScanHit:
    key: int
    offset: int
    kind: int
    compressed: bool


class Engine:
    """One device context (kh_open).  Not thread-safe; one Engine per GPU."""

    def __init__(self, device: int = 0, lanes: int = 0, groups_per_launch: int = 0):
        self._ctx = ctypes.c_void_p()
        r = lib().kh_open(device, ctypes.byref(self._ctx))
        if r:
            raise KhError(f"kh_open({device}) failed: {lib().kh_strerror(r).decode()}")
        self.device = device
        if lanes or groups_per_launch:
            self.set_geometry(lanes, groups_per_launch)

    # -- plumbing ------------------------------------------------------------------------------
    def _chk(self, r: int, what: str) -> None:
        if r:
            raise KhError(f"{what}: {lib().kh_strerror(r).decode()} ({lib().kh_last_error(self._ctx).decode()})")

    def close(self) -> None:
        if self._ctx:
            lib().kh_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_geometry(self, lanes: int = 0, groups_per_launch: int = 0) -> None:
        self._chk(lib().kh_set_geometry(self._ctx, lanes, groups_per_launch), "kh_set_geometry")

    def bsgs_geometry(self) -> tuple[int, float, float]:
        """(lanes kept for large BSGS calls or 0, giant points/s of the pad placement kept, of the best
        other candidate) -- the context's placement calibration (kh_bsgs_geometry)."""
        lanes, rates = ctypes.c_uint32(), (ctypes.c_double * 2)()
        self._chk(lib().kh_bsgs_geometry(self._ctx, ctypes.byref(lanes), ctypes.byref(rates)), "kh_bsgs_geometry")
        return lanes.value, rates[0], rates[1]

    def debug_layout(self) -> dict:
        """Device addresses and sizes of layer 1, the inversion pad and layer 2 (kh_debug_layout)."""
        o = (ctypes.c_uint64 * 8)()
        self._chk(lib().kh_debug_layout(self._ctx, ctypes.byref(o)), "kh_debug_layout")
        return {"layer1": [hex(o[0]), o[1]], "pad": [hex(o[2]), o[3]], "layer2": [hex(o[4]), o[5]],
                "lanes": o[6], "pad_rows": o[7]}

    def debug_replace(self, which: int) -> None:
        """Give device buffers fresh allocations (kh_debug_replace; diagnostics): 1 layer 1, 2 the pad,
        4 the lane arrays, 8 the delta tables, 16 layers 2 and 3."""
        self._chk(lib().kh_debug_replace(self._ctx, which), "kh_debug_replace")

    def debug_burn(self, ms: float) -> None:
        """Enqueue ~ms of VALU-dense load on the walk's stream (kh_debug_burn; diagnostics)."""
        self._chk(lib().kh_debug_burn(self._ctx, ms), "kh_debug_burn")

    def debug_replace_layer1(self) -> None:
        self.debug_replace(1)

    def bsgs_placement(self) -> tuple[bool, list[float]]:
        """(calibration complete, [pad kept, pad other, layer-1 kept, layer-1 other] giant points/s)."""
        rates = (ctypes.c_double * 4)()
        r = lib().kh_bsgs_placement(self._ctx, ctypes.byref(rates))
        if r < 0:
            self._chk(r, "kh_bsgs_placement")
        return r == 1, list(rates)

    def release_walk(self) -> None:
        """Free the walks' lane arrays and inversion pad (kh_release_walk)."""
        self._chk(lib().kh_release_walk(self._ctx), "kh_release_walk")

    def set_rmd_batch(self, group: int) -> None:
        """-m rmd160 --rmd-batch-size: the reference's clamped group size (1024 = the ordinary walk)."""
        self._chk(lib().kh_set_rmd_batch(self._ctx, group), "kh_set_rmd_batch")

    def synchronize(self) -> None:
        self._chk(lib().kh_synchronize(self._ctx), "kh_synchronize")

    # -- address / rmd160 / xpoint -------------------------------------------------------------
    def set_targets(self, rows: list[bytes], bloom_items: int = 0) -> None:
        buf = b"".join(rows)
        assert all(len(r) == 20 for r in rows)
        self._chk(lib().kh_set_targets(self._ctx, buf, len(rows), bloom_items), "kh_set_targets")

    def set_vanity(self, ranges: list[tuple[bytes, bytes]], probe_len: int, bloom_items: int = 0) -> None:
        """Vanity prefixes (kh_set_vanity): hash160 ranges [A, B], the bloom keyed on A's first probe_len bytes."""
        assert all(len(a) == 20 and len(b) == 20 for a, b in ranges)
        buf = b"".join(a + b for a, b in ranges)
        self._chk(lib().kh_set_vanity(self._ctx, buf, len(ranges), probe_len, bloom_items), "kh_set_vanity")

    def targets_save(self, path: str) -> None:
        """Write the -S target file (data_<hex>.dat layout) of the current targets to path."""
        self._chk(lib().kh_targets_save(self._ctx, path.encode()), "kh_targets_save")

    def targets_load(self, path: str, skip_checksum: bool = False) -> None:
        """Targets (rows and bloom, geometry included) from a data_<hex>.dat file, instead of set_targets."""
        self._chk(lib().kh_targets_load(self._ctx, path.encode(), 1 if skip_checksum else 0), "kh_targets_load")

    def scan(self, start: int, n_keys: int, mode: int = KH_MODE_ADDRESS, search: int = KH_SEARCH_BOTH,
             stride: int = 1, cap: int = 4096, endo: bool = False) -> list[ScanHit]:
        """endo: -e (also the endomorphism images; hit kinds then carry KH_KIND_ENDO1/2, KH_KIND_NEGY)."""
        hits = (KhHit * cap)()
        n = ctypes.c_uint32(0)
        r = lib().kh_scan(self._ctx, be32(start), be32(stride), n_keys, mode | (KH_MODE_ENDO if endo else 0), search,
                          hits, cap, ctypes.byref(n))
        self._chk(r, "kh_scan")
        return [ScanHit(int.from_bytes(bytes(h.key), "big"), h.offset, h.kind, bool(h.compressed))
                for h in hits[: n.value]]

    def scan_status(self, start: int, n_keys: int, mode: int = KH_MODE_ADDRESS, search: int = KH_SEARCH_BOTH,
                    stride: int = 1, cap: int = 4096) -> tuple[int, list[ScanHit]]:
        """kh_scan returning (status, hits) instead of raising: a KH_E_RANGE call (--rmd-batch-size, a
        group centred on the key 0 mod n) still returns the hits of the groups before it."""
        hits = (KhHit * cap)()
        n = ctypes.c_uint32(0)
        r = lib().kh_scan(self._ctx, be32(start), be32(stride), n_keys, mode, search, hits, cap, ctypes.byref(n))
        return r, [ScanHit(int.from_bytes(bytes(h.key), "big"), h.offset, h.kind, bool(h.compressed))
                   for h in hits[: min(n.value, cap)]]

    # -- BSGS ----------------------------------------------------------------------------------
    def bsgs_setup(self, n: int, k: int, layer1: int = None) -> KhBsgsInfo:
        """layer1: KH_LAYER1_BLOCKED (default) or KH_LAYER1_REFERENCE (bit-identical to the reference)."""
        if layer1 is not None:
            self._chk(lib().kh_bsgs_set_layer1(self._ctx, layer1), "kh_bsgs_set_layer1")
        info = KhBsgsInfo()
        self._chk(lib().kh_bsgs_setup(self._ctx, n, k, ctypes.byref(info)), "kh_bsgs_setup")
        return info

    def bsgs_build(self) -> None:
        self._chk(lib().kh_bsgs_build(self._ctx), "kh_bsgs_build")

    def bsgs_save(self, directory: str) -> None:
        """Write the -S table files (keyhunt_bsgs_{4,6,7}_*.blm, keyhunt_bsgs_2_*.tbl) into directory."""
        self._chk(lib().kh_bsgs_save(self._ctx, directory.encode()), "kh_bsgs_save")

    def bsgs_load(self, directory: str, skip_checksum: bool = False) -> None:
        """Load the -S table files instead of bsgs_build (after bsgs_setup)."""
        self._chk(lib().kh_bsgs_load(self._ctx, directory.encode(), 1 if skip_checksum else 0), "kh_bsgs_load")

    def bsgs_set_targets(self, points: list[tuple[int, int]]) -> None:
        buf = b"".join(be32(x) + be32(y) for x, y in points)
        self._chk(lib().kh_bsgs_set_targets(self._ctx, buf, len(points)), "kh_bsgs_set_targets")

    def bsgs_scan(self, start: int, n_bases: int, cap: int = 1024) -> list[tuple[int, int]]:
        out = (KhBsgsFound * cap)()
        n = ctypes.c_uint32(0)
        self._chk(lib().kh_bsgs_scan(self._ctx, be32(start), n_bases, out, cap, ctypes.byref(n)), "kh_bsgs_scan")
        return [(f.target, int.from_bytes(bytes(f.key), "big")) for f in out[: n.value]]

    def bsgs_scan_list(self, bases: list[int], cap: int = 1024) -> list[tuple[int, int]]:
        """Scan an arbitrary list of bases (each walks its own 2N keys)."""
        out = (KhBsgsFound * cap)()
        n = ctypes.c_uint32(0)
        buf = b"".join(be32(b) for b in bases)
        self._chk(lib().kh_bsgs_scan_list(self._ctx, buf, len(bases), out, cap, ctypes.byref(n)), "kh_bsgs_scan_list")
        return [(f.target, int.from_bytes(bytes(f.key), "big")) for f in out[: n.value]]

    def bsgs_reset_found(self) -> None:
        self._chk(lib().kh_bsgs_reset_found(self._ctx), "kh_bsgs_reset_found")

    def bsgs_candidates(self) -> int:
        c = ctypes.c_uint64()
        self._chk(lib().kh_bsgs_candidates(self._ctx, ctypes.byref(c)), "kh_bsgs_candidates")
        return c.value

    def bsgs_refine_stats(self) -> tuple[int, int]:
        """(first-level candidates, layer-2 hits of their second checks) since bsgs_setup."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(lib().kh_bsgs_refine_stats(self._ctx, ctypes.byref(a), ctypes.byref(b)), "kh_bsgs_refine_stats")
        return a.value, b.value

    def bsgs_log_candidates(self, enable: bool = True) -> None:
        self._chk(lib().kh_bsgs_log_candidates(self._ctx, int(enable)), "kh_bsgs_log_candidates")

    def bsgs_logged_candidates(self) -> list[tuple[int, int, int]]:
        """(base ordinal, a, layer-2 mask) of every first-level candidate since bsgs_log_candidates."""
        n = ctypes.c_uint64()
        lib().kh_bsgs_get_candidates(self._ctx, None, None, None, ctypes.c_uint64(0), ctypes.byref(n))
        m = max(n.value, 1)
        b, a, k = (ctypes.c_uint64 * m)(), (ctypes.c_uint32 * m)(), (ctypes.c_uint32 * m)()
        self._chk(lib().kh_bsgs_get_candidates(self._ctx, b, a, k, ctypes.c_uint64(m), ctypes.byref(n)),
                  "kh_bsgs_get_candidates")
        return [(b[i], a[i], k[i]) for i in range(n.value)]

    def bsgs_second_masks(self, target: int, base_keys: list[int]) -> tuple[list[int], list[int]]:
        """(GPU, host) layer-2 masks of bsgs_secondcheck for each base key (parity hook)."""
        n = len(base_keys)
        buf = b"".join(be32(k) for k in base_keys) or bytes(32)
        g, h = (ctypes.c_uint32 * max(n, 1))(), (ctypes.c_uint32 * max(n, 1))()
        self._chk(lib().kh_bsgs_second_masks(self._ctx, target, buf, n, g, h), "kh_bsgs_second_masks")
        return list(g[:n]), list(h[:n])

    # -- measurement ---------------------------------------------------------------------------
    def kernel_time(self, kind: int) -> tuple[int, float, int]:
        la, ms, pts = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        self._chk(lib().kh_kernel_time(self._ctx, kind, ctypes.byref(la), ctypes.byref(ms), ctypes.byref(pts)),
                  "kh_kernel_time")
        return la.value, ms.value, pts.value

    def kernel_time_reset(self) -> None:
        self._chk(lib().kh_kernel_time_reset(self._ctx), "kh_kernel_time_reset")

    # -- parity hooks --------------------------------------------------------------------------
    def pubkeys(self, scalars: list[int]) -> list[tuple[int, int]]:
        buf = b"".join(be32(s) for s in scalars)
        out = ctypes.create_string_buffer(64 * len(scalars))
        self._chk(lib().kh_pubkeys(self._ctx, buf, len(scalars), out), "kh_pubkeys")
        raw = out.raw
        return [(int.from_bytes(raw[64 * i:64 * i + 32], "big"), int.from_bytes(raw[64 * i + 32:64 * i + 64], "big"))
                for i in range(len(scalars))]

    def walk_points(self, start: int, n_points: int, stride: int = 1, need_y: bool = False):
        xs = ctypes.create_string_buffer(32 * n_points)
        ys = ctypes.create_string_buffer(32 * n_points) if need_y else None
        self._chk(lib().kh_walk_points(self._ctx, be32(start), be32(stride), n_points, xs, ys), "kh_walk_points")
        return xs.raw, (ys.raw if need_y else None)

    def hash160(self, points: list[tuple[int, int]]) -> list[tuple[bytes, bytes, bytes]]:
        buf = b"".join(be32(x) + be32(y) for x, y in points)
        out = ctypes.create_string_buffer(60 * len(points))
        self._chk(lib().kh_hash160(self._ctx, buf, len(points), out), "kh_hash160")
        raw = out.raw
        return [(raw[60 * i:60 * i + 20], raw[60 * i + 20:60 * i + 40], raw[60 * i + 40:60 * i + 60])
                for i in range(len(points))]

    def field_ops(self, a: list[int], b: list[int]) -> list[tuple[int, int, int, int, int]]:
        ba = b"".join(be32(x) for x in a)
        bb = b"".join(be32(x) for x in b)
        out = ctypes.create_string_buffer(160 * len(a))
        self._chk(lib().kh_field_ops(self._ctx, ba, bb, len(a), out), "kh_field_ops")
        raw = out.raw
        return [tuple(int.from_bytes(raw[160 * i + 32 * k:160 * i + 32 * k + 32], "big") for k in range(5))
                for i in range(len(a))]

    def bloom_check(self, layer: int, items: list[bytes]) -> list[bool]:
        ln = len(items[0])
        out = ctypes.create_string_buffer(len(items))
        self._chk(lib().kh_bloom_check(self._ctx, layer, b"".join(items), len(items), ln, out), "kh_bloom_check")
        return [b != 0 for b in out.raw]

    def get_bloom(self, layer: int) -> bytes:
        nb = ctypes.c_uint64()
        self._chk(lib().kh_get_bloom(self._ctx, layer, None, 0, ctypes.byref(nb)), "kh_get_bloom")
        buf = ctypes.create_string_buffer(nb.value)
        self._chk(lib().kh_get_bloom(self._ctx, layer, buf, nb.value, ctypes.byref(nb)), "kh_get_bloom")
        return buf.raw

    def get_bsgs_table(self) -> bytes:
        n = ctypes.c_uint64()
        self._chk(lib().kh_get_bsgs_table(self._ctx, None, 0, ctypes.byref(n)), "kh_get_bsgs_table")
        buf = ctypes.create_string_buffer(16 * n.value)
        self._chk(lib().kh_get_bsgs_table(self._ctx, buf, n.value, ctypes.byref(n)), "kh_get_bsgs_table")
        return buf.raw

    def set_bsgs_table(self, rows: bytes) -> None:
        """--load-ptable: use these 16-byte rows as the bP table (keyhunt.cpp:1871-1892)."""
        self._chk(lib().kh_bsgs_set_table(self._ctx, rows, len(rows) // 16), "kh_bsgs_set_table")
