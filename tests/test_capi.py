"""The C ABI library loads on a CPU-only host and exports exactly what include/kh_gpu.h declares;
host-side argument checking works without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

import keyhunt_amd
from keyhunt_amd import engine as E


def test_library_exports_every_header_symbol():
    L = keyhunt_amd.lib()
    syms = keyhunt_amd.header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s


def test_abi_version_and_errors():
    L = keyhunt_amd.lib()
    assert L.kh_abi_version() == 1
    assert L.kh_strerror(0) == b"ok"
    assert L.kh_strerror(-6).startswith(b"BSGS n")


def test_null_context_is_rejected():
    L = keyhunt_amd.lib()
    n = ctypes.c_uint32()
    assert L.kh_scan(None, b"\0" * 32, None, 1024, 0, 0, None, 0, ctypes.byref(n)) == -1
    assert L.kh_bsgs_setup(None, 1 << 20, 1, None) == -1
    assert L.kh_open(0, None) == -1


def test_device_count_without_gpu_is_zero_or_more():
    assert keyhunt_amd.device_count() >= 0


def test_cli_rejects_out_of_scope_and_bad_nk(tmp_path):
    cli = os.path.join(E.PKG, "bin", "keyhunt-amd")
    if not os.path.exists(cli):
        pytest.skip("CLI not built")
    r = subprocess.run([cli, "-m", "minikeys", "-f", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "Unsupported mode" in r.stderr
    r = subprocess.run([cli, "-m", "address", "-f", "x", "-r", "1:100000", "-n", "0x10000"], capture_output=True,
                       text=True)
    assert r.returncode == 1 and "n must be at least 2^20" in r.stderr
    r = subprocess.run([cli, "-m", "bsgs", "-f", "x", "-k", "5000", "-b", "66"], capture_output=True, text=True)
    assert r.returncode == 1 and "too large" in r.stderr
    r = subprocess.run([cli, "-m", "address", "-f", "x", "-S"], capture_output=True, text=True)
    assert r.returncode == 1   # -S is accepted, the missing target file is not
    # -B ggsb and its long options are accepted (the missing file / GPU is what fails here)
    r = subprocess.run([cli, "-m", "bsgs", "-f", "x", "-B", "ggsb", "--bsgs-block-count", "4"], capture_output=True,
                       text=True)
    assert r.returncode == 1 and "ggsb" not in r.stderr
    r = subprocess.run([cli, "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "Usage" in r.stdout
    r = subprocess.run([cli, "-m", "rmd160", "-f", "x", "-z", "2", "-r", "1:100000"], capture_output=True, text=True)
    assert "Bloom Size Multiplier 2" in r.stdout
    # keyhunt.cpp:1185-1193 test the -B index against MODE_BSGS: -B both + -e / -I fail in any mode
    r = subprocess.run([cli, "-m", "address", "-f", "x", "-B", "both", "-e"], capture_output=True, text=True)
    assert r.returncode == 1 and "Endomorphism doesn't work with BSGS" in r.stderr
    r = subprocess.run([cli, "-m", "address", "-f", "x", "-B", "both", "-I", "3"], capture_output=True, text=True)
    assert r.returncode == 1 and "Stride doesn't work with BSGS" in r.stderr


ORDER = "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141"


def test_cli_range_forms(tmp_path):
    """-r START[:END] and the defaults (keyhunt.cpp:1024-1055, 1221-1255, 1534-1540): START alone runs
    to the group order; no range walks 1..order (address family) or a random start..order (BSGS);
    an unusable range falls back to those defaults with the reference's messages."""
    cli = os.path.join(E.PKG, "bin", "keyhunt-amd")
    if not os.path.exists(cli):
        pytest.skip("CLI not built")

    def rng(*argv):
        r = subprocess.run([cli, "-m", "xpoint", "-f", "x"] + list(argv), capture_output=True, text=True)
        m = re.search(r"-- from : 0x([0-9a-fA-F]+)\n\[\+\] -- to   : 0x([0-9a-fA-F]+)", r.stdout)
        return (m.group(1).lower(), m.group(2).lower()) if m else None, r.stderr

    assert rng("-r", "7cce5efdac000000")[0] == ("7cce5efdac000000", ORDER)
    assert rng("-r", "10:20")[0] == ("10", "20")
    got, err = rng("-r", "20:10")
    assert got == ("10", "20") and "Swapping them" in err
    assert rng("-r", "0:20")[0] == ("1", "20")  # start 0 is bumped to 1
    assert rng()[0] == ("1", ORDER)
    got, err = rng("-r", "5:5")
    assert got == ("1", ORDER) and "can't be the same" in err
    got, err = rng("-r", "zz:10")
    assert got == ("1", ORDER) and "Invalid hexstring : zz" in err
    # BSGS reads its targets before printing a range, and prints none for a random start
    # (keyhunt.cpp:1367-1372, 1517-1540): here the missing file is what fails
    r = subprocess.run([cli, "-m", "bsgs", "-f", "x"], capture_output=True, text=True)
    assert "-- to   : 0x" not in r.stdout and "Can't open file x" in r.stderr


def test_cli_vanity_and_eth_argument_checks(tmp_path):
    cli = os.path.join(E.PKG, "bin", "keyhunt-amd")
    if not os.path.exists(cli):
        pytest.skip("CLI not built")
    r = subprocess.run([cli, "-m", "vanity", "-r", "1:100000", "-v", "1Bitc0in", "-f", str(tmp_path / "none.txt")],
                       capture_output=True, text=True)
    assert 'The string "1Bitc0in" is not Valid Base58' in r.stderr and r.returncode == 1
    r = subprocess.run([cli, "-m", "address", "-c", "doge", "-f", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "Unknow crypto value doge" in r.stderr
    # -e -c eth is accepted (the reference runs it, keyhunt.cpp:3524-3536); no GPU is what fails here
    r = subprocess.run([cli, "-m", "address", "-c", "eth", "-e", "-f", "x"], capture_output=True, text=True)
    assert "-e with -c eth" not in r.stderr and "Setting search for ETH" in r.stdout


def test_bsgsd_rejects_bad_arguments_before_any_gpu_call():
    d = os.path.join(E.PKG, "bin", "bsgsd-amd")
    if not os.path.exists(d):
        pytest.skip("bsgsd-amd not built")
    r = subprocess.run([d, "-n", "0x10000"], capture_output=True, text=True)
    assert r.returncode == 1 and "n must be at least 2^20" in r.stderr
    r = subprocess.run([d, "-n", "0x1000000", "-k", "5"], capture_output=True, text=True)
    assert r.returncode == 1 and "too large" in r.stderr
    r = subprocess.run([d, "-B", "random"], capture_output=True, text=True)
    assert r.returncode == 1 and "sequentially" in r.stderr
    r = subprocess.run([d, "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "usage" in r.stdout


def test_cli_ptable_flags_parse(tmp_path):
    """--ptable / --ptable-size / --load-ptable / --ptable-cache are accepted (keyhunt.cpp:772-789);
    --load-ptable alone fails with the reference's message (1126-1129)."""
    cli = os.path.join(E.PKG, "bin", "keyhunt-amd")
    if not os.path.exists(cli):
        pytest.skip("CLI not built")
    r = subprocess.run([cli, "-m", "bsgs", "-f", "x", "--load-ptable"], capture_output=True, text=True)
    assert r.returncode == 1 and "--load-ptable requires --ptable <file>" in r.stderr
    # with a readable target file the run gets as far as looking for a device (none here)
    import shutil
    shutil.copy(os.path.join(os.path.dirname(__file__), "golden", "data", "63.pub"), tmp_path)
    r = subprocess.run([cli, "-m", "bsgs", "-f", "63.pub", "-r", "7cce5a0000000000:7cce9a0000000000", "--ptable", "t",
                        "--ptable-size", "1m", "--load-ptable", "--ptable-cache"], capture_output=True, text=True,
                       cwd=tmp_path, env=dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1"))
    assert r.returncode == 1 and "ptable" not in r.stderr and "no GPU found" in r.stderr


def test_host_md5_matches_hashlib(tmp_path):
    """The CLI's RFC 1321 MD5 (host/kh_host_util.h, for --ptable-cache) against hashlib."""
    import hashlib
    import shutil
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = tmp_path / "m.cpp"
    src.write_text('#include "kh_host_util.h"\nint main(int, char **v) { uint8_t o[16];\n'
                   '  if (!khh::md5_of_file(v[1], o)) return 1;\n'
                   '  for (int i = 0; i < 16; i++) printf("%02x", o[i]); return 0; }\n')
    exe = tmp_path / "m"
    inc = os.path.join(os.path.dirname(E.PKG), "include")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(E.PKG, "host"), "-I", inc, "-o", str(exe),
                    str(src)], check=True)
    for n in (0, 1, 55, 56, 63, 64, 65, 1000, (1 << 20) + 17):
        data = bytes((i * 131 + n) & 0xFF for i in range(n))
        f = tmp_path / f"d{n}"
        f.write_bytes(data)
        out = subprocess.run([str(exe), str(f)], capture_output=True, text=True, check=True).stdout
        assert out == hashlib.md5(data).hexdigest(), n


def test_scan_memory_figures():
    """kh_scan_memory (context-free, no device call): a 2^32-key chunk of -m address/rmd160 holds 2^20
    lanes x 4096-point groups of 32-B pad rows (64 GiB), -m xpoint's sparse pad half of that, -e and
    the small-group walks (a chunk that is no multiple of 4096 keys) the dense 1024-point pad."""
    import ctypes
    from keyhunt_amd.engine import lib
    def need(n, mode, search):
        v = ctypes.c_uint64(0)
        assert lib().kh_scan_memory(n, mode, search, ctypes.byref(v)) == 0
        return v.value
    pad = (1 << 20) * 2048 * 32
    assert pad <= need(1 << 32, 0, 0) < pad + (1 << 30)
    assert pad // 2 <= need(1 << 32, 1, 0) < pad // 2 + (1 << 30)
    assert need(1 << 32, 0, 2) < pad  # -l both: 1024-point groups, 2^18 lanes
    assert lib().kh_scan_memory(0, 0, 0, ctypes.byref(ctypes.c_uint64())) != 0
