"""-S target caches for -m address|rmd160|xpoint (and -c eth): data_<hex>.dat, written by
writeFileIfNeeded (keyhunt.cpp:7756-7855) and read by readFileAddress (7033-7210).

tests/golden/ref_data/ holds the files the reference CLI wrote for four target files
(oracle/make_golden.py --data) with their sizes, digests (struct bloom heap pointer masked) and the
keys that run found.  The engine's CLI must write the same bytes, read its own and the reference's
files back with the same hits, and reject a corrupted file unless -6 skips the checksums.  One case
has 12032 rows and -z 2, so its bloom is sized past the 10000-entry floor (keyhunt.cpp:7608)."""
import hashlib
import json
import os
import shutil
import subprocess
import tempfile

import pytest

from _cli import CLI, parse_keyfound
from conftest import DATA, GOLDEN

pytestmark = pytest.mark.gpu
REFD = os.path.join(GOLDEN, "ref_data")
INDEX = json.load(open(os.path.join(REFD, "index.json")))
CASES = sorted(k for k in INDEX if not k.startswith("_"))


def masked_digest(path):
    data = bytearray(open(path, "rb").read())
    data[32 + 64: 32 + 72] = bytes(8)  # struct bloom `bf`: the reference's heap pointer
    return hashlib.sha256(bytes(data)).hexdigest()


def run_in(td, argv, timeout=300):
    kf = os.path.join(td, "KEYFOUNDKEYFOUND.txt")
    if os.path.exists(kf):
        os.remove(kf)
    p = subprocess.run([CLI] + argv + ["-q", "-s", "0"], cwd=td, capture_output=True, text=True, timeout=timeout)
    hits = parse_keyfound(open(kf).read()) if os.path.exists(kf) else []
    return p, sorted({h["key"] for h in hits})


def fresh_dir(case):
    td = tempfile.mkdtemp()
    src = INDEX[case]["source"]
    if src == "many.rmd":  # > 10000 rows, generated (tests/golden/make_many_targets.py)
        import sys
        sys.path.insert(0, GOLDEN)
        import make_many_targets
        make_many_targets.write(os.path.join(td, src))
    else:
        shutil.copy(os.path.join(DATA, src), td)
    return td


@pytest.mark.parametrize("case", CASES)
def test_written_data_file_equals_reference_and_reads_back(case):
    want = INDEX[case]
    argv = want["argv"][:want["argv"].index("-t")]
    td = fresh_dir(case)
    try:
        p, keys = run_in(td, argv)
        assert p.returncode == 0, p.stderr
        assert f"Writing file {want['file']}" in p.stdout
        path = os.path.join(td, want["file"])
        assert os.path.getsize(path) == want["size"]
        assert masked_digest(path) == want["masked_sha256"]
        assert keys == sorted(want["keys"])
        p2, keys2 = run_in(td, argv)           # second run: reads the cache
        assert p2.returncode == 0, p2.stderr
        assert f"Reading file {want['file']}" in p2.stdout and "Writing file" not in p2.stdout
        assert keys2 == keys
    finally:
        shutil.rmtree(td)


@pytest.mark.parametrize("case", [c for c in CASES if INDEX[c].get("committed", True)])
def test_reads_reference_written_data_file(case):
    want = INDEX[case]
    argv = want["argv"][:want["argv"].index("-t")]
    td = fresh_dir(case)
    try:
        shutil.copy(os.path.join(REFD, want["file"]), td)
        p, keys = run_in(td, argv)
        assert p.returncode == 0, p.stderr
        assert f"Reading file {want['file']}" in p.stdout
        assert keys == sorted(want["keys"])
    finally:
        shutil.rmtree(td)


def test_corrupted_data_file_rejected_unless_checksums_skipped():
    want = INDEX["rmd160_1to32"]
    argv = want["argv"][:want["argv"].index("-t")]
    td = fresh_dir("rmd160_1to32")
    try:
        path = os.path.join(td, want["file"])
        data = bytearray(open(os.path.join(REFD, want["file"]), "rb").read())
        data[32 + 112 + 100] ^= 0x01            # one bloom bit flipped: sha256(bits) mismatch
        open(path, "wb").write(bytes(data))
        p, _ = run_in(td, argv)
        assert p.returncode != 0 and "checksum" in p.stderr
        p, keys = run_in(td, argv + ["-6"])     # FLAGSKIPCHECKSUM: the file is used as is
        assert p.returncode == 0, p.stderr
        assert keys == sorted(want["keys"])
    finally:
        shutil.rmtree(td)


def test_engine_load_uses_file_bloom_and_rows(engine):
    """kh_targets_load takes the bloom bits and the rows from the file: the target bloom read back
    equals the file's bit array, and a save writes the same bytes again."""
    want = INDEX["xpoint_1to63_65"]
    src = os.path.join(REFD, want["file"])
    raw = open(src, "rb").read()
    nbytes = int.from_bytes(raw[32 + 16:32 + 24], "little")
    engine.targets_load(src)
    assert engine.get_bloom(0) == raw[32 + 112:32 + 112 + nbytes]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "x.dat")
        engine.targets_save(out)
        assert masked_digest(out) == want["masked_sha256"]
