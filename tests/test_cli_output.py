"""CPU checks of the output-contract fixtures (tests/golden/ref_stdout.json) and of the rule the CLI
uses for in-place progress lines: a run of "\\r<line>\\r" writes shows on a terminal as their overlay,
so printing the overlay once per engine call (keyhunt_cli.cpp base_lines) renders exactly what the
reference's per-base writes render (keyhunt.cpp:4626-4631, 3340-3345)."""
import json
import os
import re

from conftest import GOLDEN
from _cli import render, run_section

REF = json.load(open(os.path.join(GOLDEN, "ref_stdout.json")))


def overlay(lines: list[str]) -> str:
    out = ""
    for ln in lines:
        out = ln if len(ln) >= len(out) else ln + out[len(ln):]
    return out


def collapse(text: str) -> str:
    """Every run of consecutive in-place lines replaced by one write of their overlay."""
    def sub(m):
        return "\r" + overlay(re.findall(r"\r([^\r\n]*)\r", m.group(0))) + "\r"
    return re.sub(r"(?:\r[^\r\n]*\r)+", sub, text)


def test_fixtures_present():
    names = {k for k in REF if not k.startswith("_")}
    for n in ("rmd160_M", "rmd160_verbose", "bsgs_63_M", "bsgs_63_verbose", "bsgs_two_verbose", "rmd160_stats_M"):
        assert n in names


def test_overlay_renders_like_every_line():
    for name, ref in REF.items():
        if name.startswith("_") or "stdout" not in ref:
            continue
        sec = run_section(ref["stdout"])
        assert sec, name
        assert render(collapse(sec)) == render(sec), name


def test_overlay_of_shrinking_lines():
    s = "\r[+] Thread 0x10000   \r\r[+] Thread 0xffff   \r"
    assert render(collapse(s)) == render(s) == "[+] Thread 0xffff    "


def test_matrix_lines_one_per_base():
    """-M: one "[+] Thread 0x<base> \\n" per base up to the one holding the key, then the key."""
    sec = run_section(REF["bsgs_63_bases_M"]["stdout"])
    bases = re.findall(r"\[\+\] Thread 0x([0-9a-f]+) \n", sec)
    assert [int(b, 16) for b in bases] == [0x7cce5efdac000000 + i * 0x200000 for i in range(7)]
    assert sec.endswith("[+] Thread Key found privkey 7cce5efdaccf6808   [+] Publickey "
                        "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579\nAll points were found\n")


def test_stats_fixture_terminators():
    assert all(l.endswith("\n") and not l.startswith("\r") for l in REF["rmd160_stats_M"]["stats_lines"])
    assert all(l.startswith("\r") and l.endswith("\r") for l in REF["rmd160_stats"]["stats_lines"])


def _header_lines(text: str, upto_n: bool = False) -> list[str]:
    """The lines before the run section, without the version line (the engine's own).  upto_n: for
    BSGS only up to "[+] N = ..." -- what the CLI prints before it opens a device; the table-setup
    lines after it (keyhunt.cpp:1687-1845, 2225-2503) come from the first context's worker and are
    compared on the GPU (tests/test_gpu_stdout.py)."""
    m = __import__("_cli").RUN_START.search(text)
    lines = [l for l in (text[:m.start()] if m else text).split("\n") if l and not l.startswith("[+] Version")]
    if upto_n:
        lines = lines[:next(i for i, l in enumerate(lines) if l.startswith("[+] N = ")) + 1]
    return lines


def test_cli_header_matches_reference():
    """keyhunt-amd prints the reference's header lines (option echoes, mode, N, range, target loading)
    in the reference's order, before it looks for a GPU: run here with no device, it stops right after
    them ("[E] no GPU found")."""
    import shutil
    import subprocess
    import tempfile
    from conftest import DATA
    from _cli import CLI
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    for name, ref in REF.items():
        if name.startswith("_") or "stdout" not in ref:
            continue
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            p = subprocess.run([CLI] + ref["argv"] + ["-t", "1", "-s", "0"], cwd=td, capture_output=True, text=True,
                               timeout=60, env=env)
        bsgs = "bsgs" in ref["argv"]
        got = _header_lines(p.stdout, bsgs)
        assert got == _header_lines(ref["stdout"], bsgs), name


def test_bsgs_setup_lines_model():
    """The table-setup lines the CLI prints for BSGS (keyhunt_cli.cpp print_layer_lines /
    print_allocating / print_build_lines), restated here from M alone, equal the reference CLI's on
    every BSGS fixture: the per-layer element counts, per-shard bloom_init2 sizes, float layer totals,
    the bP allocation, the single-thread progress lines, checksums and sort."""
    import math
    def init2_bytes(entries):
        bpe = -math.log(1e-6) / 0.480453013918201
        bits = int(entries * bpe)
        return bits // 8 + (1 if bits % 8 else 0)
    import struct
    def f32(x):
        return struct.unpack("f", struct.pack("f", x))[0]
    runs = [(n, r) for n, r in REF.items() if not n.startswith("_") and "stdout" in r]
    runs += [(n, r) for n, v in REF.items() if not n.startswith("_") and "seq" in v for r in v["seq"]]
    for name, ref in runs:
        if "bsgs" not in ref["argv"] or "-S" in ref["argv"] or "--ptable" in ref["argv"]:
            continue
        head = _header_lines(ref["stdout"])
        n = int(head[next(i for i, l in enumerate(head) if l.startswith("[+] N = "))].split("0x")[1], 16)
        k = int(ref["argv"][ref["argv"].index("-k") + 1]) if "-k" in ref["argv"] else 1
        z = int(ref["argv"][ref["argv"].index("-z") + 1]) if "-z" in ref["argv"] else 1
        m = math.isqrt(n) * k
        m2 = -(-m // 32)
        m3 = -(-m2 // 32)
        want = []
        for ml, fl in ((m, 10000), (m2, 1000), (m3, 1000)):
            items = ml // 256 + (1 if ml % 256 else 0) if ml // 256 > fl else 1000
            b = init2_bytes(10000 if items <= 10000 else z * items)
            shard = [f"[+] Bloom filter for {items} elements.", f"[+] Loading data to the bloomfilter total: {b / 1048576:.2f} MB"]
            want += [f"[+] Bloom filter for {ml} elements " + shard[0], shard[1]] + shard * 255
            want += [f": {f32(f32(256 * b) / 1048576.0):.2f} MB"]
        want.append(f"[+] Allocating {float(m3 * 16 // 1048576):.2f} MB for {m3} bP Points")
        w = min(1048576, m)
        units = m // w + (1 if m % w else 0)
        cnt = lambda f: f"\r[+] processing {f}/{m} bP points : {int(f / m * 100)}%\r"
        want.append(cnt(0) + "".join(cnt(u * w) for u in range(units)) + f"\r[+] processing {m}/{m} bP points : 100%     ")
        want += ["[+] Making checkums .. ... done", f"[+] Sorting {m3} elements... Done!"]
        i = next(i for i, l in enumerate(head) if l.startswith("[+] N = ")) + 1
        assert head[i:i + len(want)] == want, name
