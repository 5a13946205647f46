"""BSGS -S table files (keyhunt.cpp:2504-2652 write, 1983-2230 read) on the GPU engine.

The files the engine writes are byte-identical to the ones the reference CLI writes for the same
(n, k) -- tests/golden/ref_tables.json holds their sha256 with each struct bloom's heap pointer
masked (oracle/make_golden.py --tables) -- whatever the layer-1 layout in use.  Loading them gives
back the built tables exactly; loading files written by the reference CLI itself (oracle/_ref,
when present) does too; bad files fail with the reference's checks."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
REF = json.load(open(os.path.join(GOLDEN, "ref_tables.json")))
CASES = {"n1000000_k2": (1 << 24, 2), "n4000000_k3": (1 << 26, 3), "n100000000_k64": (1 << 32, 64)}
REF_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "keyhunt")
KEY63 = 0x7CCE5EFDACCF6808


def masked_digest(path):
    import hashlib
    data = bytearray(open(path, "rb").read())
    if path.endswith(".blm"):
        rec = len(data) // 256
        for i in range(256):
            data[i * rec + 64: i * rec + 72] = bytes(8)
    return hashlib.sha256(bytes(data)).hexdigest()


@pytest.mark.parametrize("layer1", [0, 1], ids=["reference_l1", "blocked_l1"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_saved_files_equal_reference_files(engine, case, layer1, tmp_path):
    n, k = CASES[case]
    engine.bsgs_setup(n, k, layer1=layer1)
    engine.bsgs_build()
    engine.bsgs_save(str(tmp_path))
    want = REF[case]
    got = sorted(os.listdir(tmp_path))
    assert got == sorted(want["files"])
    for f in got:
        assert os.path.getsize(tmp_path / f) == want["sizes"][f], f
        assert masked_digest(str(tmp_path / f)) == want["files"][f], f


@pytest.mark.parametrize("layer1", [0, 1], ids=["reference_l1", "blocked_l1"])
def test_load_round_trip_and_scan(engine, oracle, layer1, tmp_path):
    import keyhunt_amd as K
    n, k = CASES["n4000000_k3"]
    engine.bsgs_setup(n, k, layer1=layer1)
    engine.bsgs_build()
    built = [engine.get_bloom(l) for l in (1, 2, 3)], engine.get_bsgs_table()
    engine.bsgs_save(str(tmp_path))
    with K.Engine(0) as e:
        e.bsgs_setup(n, k, layer1=layer1)
        e.bsgs_load(str(tmp_path))
        assert ([e.get_bloom(l) for l in (1, 2, 3)], e.get_bsgs_table()) == built
        p = oracle.bsgs_params(n, k)
        e.bsgs_set_targets([oracle.pubkey(KEY63)])
        start = KEY63 - 2 * 2 * p.n - 4321
        assert e.bsgs_scan(start, 4) == [(0, KEY63)]


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref/keyhunt not built")
def test_load_files_written_by_reference_cli(oracle, tmp_path):
    import keyhunt_amd as K
    shutil.copy(os.path.join(GOLDEN, "data", "63.pub"), tmp_path)
    argv = REF["n1000000_k2"]["argv"]
    subprocess.run(["timeout", "120", REF_BIN] + argv + ["-q"], cwd=tmp_path, capture_output=True, check=False)
    n, k = CASES["n1000000_k2"]
    with K.Engine(0) as e:
        e.bsgs_setup(n, k, layer1=0)
        e.bsgs_load(str(tmp_path))
        loaded = [e.get_bloom(l) for l in (1, 2, 3)], e.get_bsgs_table()
        e.bsgs_setup(n, k, layer1=0)
        e.bsgs_build()
        assert loaded == ([e.get_bloom(l) for l in (1, 2, 3)], e.get_bsgs_table())


def test_bad_files_are_refused(engine, tmp_path):
    import keyhunt_amd as K
    n, k = CASES["n1000000_k2"]
    engine.bsgs_setup(n, k)
    engine.bsgs_build()
    engine.bsgs_save(str(tmp_path))
    # missing directory
    engine.bsgs_setup(n, k)
    with pytest.raises(K.KhError, match="missing file"):
        engine.bsgs_load(str(tmp_path / "nowhere"))
    # other geometry: the file names carry M, so n = 2^22 finds none of them
    engine.bsgs_setup(1 << 22, 2)
    with pytest.raises(K.KhError, match="missing file"):
        engine.bsgs_load(str(tmp_path))
    # a flipped bit in a layer-2 shard: checksum mismatch, accepted with the -6 skip
    f = tmp_path / "keyhunt_bsgs_6_256.blm"
    data = bytearray(f.read_bytes())
    data[112 + 1000] ^= 0x10
    f.write_bytes(bytes(data))
    engine.bsgs_setup(n, k)
    with pytest.raises(K.KhError, match="checksum"):
        engine.bsgs_load(str(tmp_path))
    engine.bsgs_setup(n, k)
    engine.bsgs_load(str(tmp_path), skip_checksum=True)
    # a header of another geometry
    data[8:16] = (12345).to_bytes(8, "little")
    f.write_bytes(bytes(data))
    engine.bsgs_setup(n, k)
    with pytest.raises(K.KhError, match="geometry"):
        engine.bsgs_load(str(tmp_path), skip_checksum=True)


def test_cli_S_writes_reference_files_then_reads_them(tmp_path):
    """keyhunt-amd -S: the first run builds and writes the files (byte-identical to the reference
    CLI's for the same argv), the second reads them; both find the key."""
    from _cli import CLI, parse_keyfound
    shutil.copy(os.path.join(GOLDEN, "data", "63.pub"), tmp_path)
    argv = [a for a in REF["n1000000_k2"]["argv"] if a not in ("-t", "4")]
    outs = []
    for run in range(2):
        kf = tmp_path / "KEYFOUNDKEYFOUND.txt"
        if kf.exists():
            kf.unlink()
        p = subprocess.run([CLI] + argv + ["-q", "-s", "0"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
        assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
        assert [h["key"] for h in parse_keyfound(kf.read_text())] == [f"{KEY63:x}"]
        outs.append(p.stdout)
        if run == 0:
            for f, d in REF["n1000000_k2"]["files"].items():
                assert masked_digest(str(tmp_path / f)) == d, f
    assert "Writing bloom filter to file keyhunt_bsgs_4_8192.blm" in outs[0]
    assert "Reading bloom filter from file keyhunt_bsgs_4_8192.blm" in outs[1]
