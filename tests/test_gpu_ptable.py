"""BSGS --ptable FILE / --ptable-size / --load-ptable (keyhunt.cpp:772-787, 1847-1956): the sorted bP
table as a raw file of M3 16-byte bsgs_xvalue rows, written by the CLI after the GPU build and read
back in place of the built rows.

The written rows are pinned by the reference's own -S file for the same argv: keyhunt_bsgs_2_<M3>.tbl
is the same rows followed by their sha256 (tests/golden/ref_tables.json).  When oracle/_ref is
present, the reference CLI's own --ptable file is compared byte for byte as well."""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
REF = json.load(open(os.path.join(GOLDEN, "ref_tables.json")))
REF_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "keyhunt")
KEY63 = 0x7CCE5EFDACCF6808
CASE = "n1000000_k2"
ARGV = [a for a in REF[CASE]["argv"] if a not in ("-t", "4", "-S")]  # -n 2^24 -k 2: M3 = 8 rows


# n = 2^32, k = 64: M3 = 4096 rows, where the third check needs the table (with 8 rows the key is
# also reached through the AMP3 special case, keyhunt.cpp:5231-5240, whatever the table holds)
BIG = ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000000", "-k", "64", "-r", "7cce5efd00000000:7cce5efe00000000"]


def _run(tmp_path, extra, argv=ARGV):
    from _cli import CLI, parse_keyfound
    kf = tmp_path / "KEYFOUNDKEYFOUND.txt"
    if kf.exists():
        kf.unlink()
    p = subprocess.run([CLI] + argv + extra + ["-q", "-s", "0"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    keys = [h["key"] for h in parse_keyfound(kf.read_text())] if kf.exists() else []
    return p, keys


@pytest.fixture
def work(tmp_path):
    shutil.copy(os.path.join(GOLDEN, "data", "63.pub"), tmp_path)
    return tmp_path


def test_ptable_file_is_the_reference_table(work):
    p, keys = _run(work, ["--ptable", "bp.tbl"])
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert keys == [f"{KEY63:x}"]
    rows = (work / "bp.tbl").read_bytes()
    tbl = [f for f in REF[CASE]["files"] if f.endswith(".tbl")][0]
    assert len(rows) + 32 == REF[CASE]["sizes"][tbl]
    assert hashlib.sha256(rows + hashlib.sha256(rows).digest()).hexdigest() == REF[CASE]["files"][tbl]


def test_ptable_size_grows_the_file_with_zeros(work):
    p, _ = _run(work, ["--ptable", "bp.tbl", "--ptable-size", "4k"])
    assert p.returncode == 1, p.stderr[-2000:]
    data = (work / "bp.tbl").read_bytes()
    assert len(data) == 4096
    assert data[128:] == bytes(4096 - 128)
    assert any(data[:128])


def test_load_ptable_uses_the_file(work):
    p, _ = _run(work, ["--ptable", "bp.tbl"], BIG)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    rows = (work / "bp.tbl").read_bytes()
    want = REF["n100000000_k64"]
    tbl = [f for f in want["files"] if f.endswith(".tbl")][0]
    assert hashlib.sha256(rows + hashlib.sha256(rows).digest()).hexdigest() == want["files"][tbl]
    # the file's rows are the table: the key is found through them...
    p, keys = _run(work, ["--ptable", "bp.tbl", "--load-ptable"], BIG)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert keys == [f"{KEY63:x}"]
    # ...and a zeroed table of the same size misses it, as the reference CLI does (exit 0, no key)
    (work / "bp.tbl").write_bytes(bytes(len(rows)))
    p, keys = _run(work, ["--ptable", "bp.tbl", "--load-ptable"], BIG)
    assert p.returncode == 0 and keys == []
    assert (work / "bp.tbl").read_bytes() == bytes(len(rows))  # mapped read-only: never rewritten


def test_load_ptable_errors(work):
    from _cli import CLI
    p = subprocess.run([CLI] + ARGV + ["--load-ptable", "-q"], cwd=work, capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "--load-ptable requires --ptable <file>" in p.stderr
    p, _ = _run(work, ["--ptable", "missing.tbl", "--load-ptable"])
    assert p.returncode == 1 and "[E] Cannot open bP table file" in p.stderr
    (work / "short.tbl").write_bytes(bytes(100))
    p, _ = _run(work, ["--ptable", "short.tbl", "--load-ptable"])
    assert p.returncode == 1 and "[E] Existing bP table file too small" in p.stderr
    # -S with --load-ptable and no .tbl (keyhunt.cpp:2180-2186; the reference CLI prints exactly this)
    p, _ = _run(work, ["--ptable", "bp.tbl"])
    p, _ = _run(work, ["-S", "--ptable", "bp.tbl", "--load-ptable"])
    assert p.returncode == 1
    assert ("[E] Missing bP table file keyhunt_bsgs_2_8.tbl\n    Remove --loadptable or generate the table first.\n"
            in p.stderr)
    assert not (work / "keyhunt_bsgs_2_8.tbl").exists()


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref/keyhunt not built")
def test_ptable_equals_reference_cli_file(work):
    ref_dir = work / "ref"
    ref_dir.mkdir()
    shutil.copy(work / "63.pub", ref_dir)
    subprocess.run(["timeout", "120", REF_BIN] + ARGV + ["-t", "4", "--ptable", "bp.tbl", "-q"], cwd=ref_dir,
                   capture_output=True, check=False)
    p, _ = _run(work, ["--ptable", "bp.tbl"])
    assert p.returncode == 1
    assert (work / "bp.tbl").read_bytes() == (ref_dir / "bp.tbl").read_bytes()
    # and the reference's file loads into the engine and finds the key
    shutil.copy(ref_dir / "bp.tbl", work / "ref.tbl")
    p, keys = _run(work, ["--ptable", "ref.tbl", "--load-ptable"])
    assert keys == [f"{KEY63:x}"]


def _cache_model(rows: bytes) -> bytes:
    """struct bptable_cache_file (keyhunt.cpp:137-143) as build_bptable_cache fills it (186-197)."""
    import struct
    m3 = len(rows) // 16
    b, pos = [], 0
    for bucket in range(256):
        while pos < m3 and rows[pos * 16] < bucket:
            pos += 1
        b.append(pos)
    b.append(m3)
    return struct.pack("<IIQ16s257Q", 0x42505443, 1, m3, hashlib.md5(rows).digest(), *b)


def test_ptable_cache_files(work):
    p, keys = _run(work, ["--ptable", "c.tbl", "--ptable-cache"], BIG)
    assert p.returncode == 1 and keys == [f"{KEY63:x}"], p.stdout[-2000:] + p.stderr[-2000:]
    assert "[I] bP table cache not found (c.tbl.cache); creating" in p.stdout
    assert "[+] bP table cache refreshed (c.tbl.cache)" in p.stdout
    rows = (work / "c.tbl").read_bytes()
    assert (work / "c.tbl.md5").read_text() == hashlib.md5(rows).hexdigest() + "\n"
    assert (work / "c.tbl.cache").read_bytes() == _cache_model(rows)
    # reload: the MD5 file is trusted and the cache hits
    p, keys = _run(work, ["--ptable", "c.tbl", "--ptable-cache", "--load-ptable"], BIG)
    assert p.returncode == 1 and keys == [f"{KEY63:x}"]
    assert "[+] bP table MD5 loaded (c.tbl.md5)" in p.stdout and "[+] bP table cache hit (c.tbl.cache)" in p.stdout
    # a cache of another MD5 is rebuilt
    bad = bytearray(_cache_model(rows))
    bad[16] ^= 1
    (work / "c.tbl.cache").write_bytes(bytes(bad))
    p, _ = _run(work, ["--ptable", "c.tbl", "--ptable-cache", "--load-ptable"], BIG)
    assert "[W] bP table cache mismatch (c.tbl.cache); rebuilding" in p.stdout
    assert (work / "c.tbl.cache").read_bytes() == _cache_model(rows)


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref/keyhunt not built")
def test_ptable_cache_equals_reference_cli_files(work):
    ref_dir = work / "ref"
    ref_dir.mkdir()
    shutil.copy(work / "63.pub", ref_dir)
    subprocess.run(["timeout", "120", REF_BIN] + BIG + ["-t", "4", "--ptable", "c.tbl", "--ptable-cache", "-q"],
                   cwd=ref_dir, capture_output=True, check=False)
    p, _ = _run(work, ["--ptable", "c.tbl", "--ptable-cache"], BIG)
    assert p.returncode == 1
    for f in ("c.tbl", "c.tbl.md5", "c.tbl.cache"):
        assert (work / f).read_bytes() == (ref_dir / f).read_bytes(), f
