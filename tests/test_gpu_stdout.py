"""The CLI's progress and stats output against the reference CLI's own stdout (SURVEY §8b "Host prints
identical strings"; tests/golden/ref_stdout.json, oracle/make_golden.py --stdout).

Single-context runs (the reference's -t 1, so its print order is deterministic) of every stdout
fixture: the "run section" of stdout -- from the first progress line or hit to the end -- equals the
reference's byte for byte with -M (keyhunt.cpp:3333-3336, 4619-4624: one line per chunk / base), and
as a terminal shows it without -M (3340-3345, 4626-4631: lines rewritten in place with \\r; the engine
prints the overlay of a call's lines once, tests/_cli.render).  The stats line keeps the reference's
shape and terminators (2904-2950): its own line with -M, rewritten in place without.  The header before
the run section -- option echoes, target loading, BSGS table-setup lines (keyhunt.cpp:1687-1845,
2225-2503) -- equals the reference's line for line; only the version line and the engine's device
count ("[+] GPUs : ...") are its own."""
import json
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from conftest import DATA, GOLDEN
from _cli import CLI, render, run_section
from test_cli_output import _header_lines

pytestmark = pytest.mark.gpu
REF = json.load(open(os.path.join(GOLDEN, "ref_stdout.json")))
RUNS = [k for k in REF if not k.startswith("_") and "stdout" in REF[k]]
STATS = [k for k in REF if not k.startswith("_") and "stats_lines" in REF[k]]


def run_raw(argv: list[str], kill_after: int | None = None, timeout: int = 300) -> subprocess.CompletedProcess:
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        cmd = [CLI] + argv
        if kill_after:
            cmd = ["timeout", "-k", "10", str(kill_after)] + cmd
        return subprocess.run(cmd, cwd=td, capture_output=True, timeout=timeout)


@pytest.mark.parametrize("name", RUNS)
def test_run_section_matches_reference(name):
    ref = REF[name]
    p = run_raw(ref["argv"] + ["-t", "1", "-s", "0", "-g", "1"])
    assert p.returncode == ref["exit"], p.stdout[-2000:] + p.stderr[-2000:]
    out = p.stdout.decode("latin-1")
    got = run_section(out)
    want = run_section(ref["stdout"])
    assert want, name
    assert render(got) == render(want)
    if "-M" in ref["argv"]:  # one line per chunk / base: the bytes themselves
        assert got == want
    # the whole header too, BSGS table-setup lines included (tests/test_cli_output.py checks the part
    # before "[+] N = " without a GPU): the engine's own lines are its version and the device count
    head = [l for l in _header_lines(out) if not l.startswith("[+] GPUs : ")]
    assert head == _header_lines(ref["stdout"])


SEQS = [k for k in REF if not k.startswith("_") and "seq" in REF[k]]


@pytest.mark.parametrize("name", SEQS)
def test_sequence_matches_reference(name):
    """Runs that share one directory (-S building then reading its table files, --mapped creating then
    reloading its shard files, --ptable with --ptable-cache then --load-ptable): each run's whole stdout
    equals the reference CLI's, the setup lines of the path it takes included."""
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        for i, ref in enumerate(REF[name]["seq"]):
            p = subprocess.run([CLI] + ref["argv"] + ["-t", "1", "-s", "0", "-g", "1"], cwd=td, capture_output=True,
                               timeout=300)
            assert p.returncode == ref["exit"], (i, p.stdout[-2000:] + p.stderr[-2000:])
            out = p.stdout.decode("latin-1")
            assert run_section(out) == run_section(ref["stdout"]), i
            head = [l for l in _header_lines(out) if not l.startswith("[+] GPUs : ")]
            assert head == _header_lines(ref["stdout"]), i


def _shape(line: str) -> str:
    return re.sub(r"[MGTPEZY]keys/s", "Xkeys/s", re.sub(r"\d+", "#", line))


@pytest.mark.parametrize("name", STATS)
def test_stats_line_shape(name):
    ref = REF[name]
    # long enough for a few 1-s stats lines, stopped after 5 s
    argv = [a if a != "1:400000000" else "1:10000000000" for a in ref["argv"]] + ["-g", "1"]
    p = run_raw(argv, kill_after=5)
    got = re.findall(r"\r?\[\+\] Total \d+ keys in \d+ seconds: [^\r\n]*[\r\n]", p.stdout.decode("latin-1"))
    assert len(got) >= 2, p.stdout[-1000:]
    assert {_shape(g) for g in got} <= {_shape(r) for r in ref["stats_lines"]} | {
        _shape(r).replace("~# Xkeys/s (# keys/s)", "# keys/s") for r in ref["stats_lines"]}
    # -M: each on a line of its own; otherwise rewritten in place
    for g in got:
        assert (g.endswith("\n") and not g.startswith("\r")) if "-M" in argv else (g.startswith("\r") and g.endswith("\r"))
