"""Helpers to run the engine's CLI (keyhunt_amd/bin/keyhunt-amd) like the reference binary and to
compare a run with a reference-CLI fixture of tests/golden/ref_e2e.json (oracle/make_golden.py)."""
import os
import re
import shutil
import subprocess
import tempfile

from conftest import DATA, REPO

CLI = os.path.join(REPO, "keyhunt_amd", "bin", "keyhunt-amd")

# the hit blocks keyhunt prints on stdout (same pattern as oracle/make_golden.py's STDOUT_BLOCK)
STDOUT_BLOCK = re.compile(r"\nHit! Private Key: [^\n]*\npubkey: [^\n]*\nAddress [^\n]*\nrmd160 [^\n]*\n"
                          r"|\n Hit!!!! Private Key: [^\n]*\naddress: [^\n]*\n"
                          r"|\nVanity Private Key: [^\n]*\npubkey: [^\n]*\nAddress [^\n]*\nrmd160 [^\n]*\n"
                          r"|\[\+\] Thread Key found privkey [0-9a-f]+ *\n?|\[\+\] Publickey [^\n]*\n")


# the reference's notes on target-file lines it skips (same pattern as oracle/make_golden.py's)
STDERR_NOTE = re.compile(r"^\[[IE]\] (?:Ommiting|Omiting|Ignoring)[^\n]*$", re.M)
STDOUT_NOTE = re.compile(r"^(?:ParsePublicKeyHex: |Invalid length: )[^\n]*$", re.M)


# where the run section of a CLI's stdout starts: the first progress line (keyhunt.cpp:3333-3346 per
# chunk, 4618-4633 per BSGS base), hit block or found line, or the final "End"
RUN_START = re.compile(r"\r?Base key: |\r?\[\+\] Thread 0x|\nHit! |\n Hit!!!! |\nVanity Private|\[\+\] Thread Key found"
                       r"|\nEnd\n")


def run_section(text: str) -> str:
    """stdout from the first progress line, hit or "End" on (the header before it is not compared)."""
    m = RUN_START.search(text)
    return text[m.start():] if m else ""


def render(text: str) -> str:
    """What a terminal shows for `text`: \\r returns to the start of the line, later characters
    overwrite earlier ones, \\n ends the line."""
    lines, cur, col = [], [], 0
    for ch in text:
        if ch == "\n":
            lines.append("".join(cur))
            cur, col = [], 0
        elif ch == "\r":
            col = 0
        else:
            if col < len(cur):
                cur[col] = ch
            else:
                cur.append(ch)
            col += 1
    lines.append("".join(cur))
    return "\n".join(lines)


def parse_keyfound(text: str, ordered: bool = False) -> list[dict]:
    """The records of KEYFOUNDKEYFOUND.txt / VANITYKEYFOUND.txt, sorted by key (or, with ordered, in
    file order per record kind, as oracle/make_golden.py stores "hits_in_order")."""
    hits = []
    for m in re.finditer(r"(Vanity )?Private Key: ([0-9a-f]+)\npubkey: ([0-9a-f]+)\nAddress (\S+)\nrmd160 ([0-9a-f]+)", text):
        h = {"key": m.group(2), "pubkey": m.group(3), "address": m.group(4), "rmd160": m.group(5)}
        if m.group(1):
            h["vanity"] = True
        hits.append(h)
    for m in re.finditer(r"Key found privkey ([0-9a-f]+)\nPublickey ([0-9a-f]+)", text):
        hits.append({"key": m.group(1), "pubkey": m.group(2)})
    for m in re.finditer(r"Private Key: ([0-9a-f]+)\naddress: (0x[0-9a-f]+)\n", text):  # writekeyeth
        hits.append({"key": m.group(1), "address": m.group(2)})
    return hits if ordered else sorted(hits, key=lambda h: int(h["key"], 16))


def run_cli(argv: list[str], timeout: int = 600, kill_after: int | None = None):
    """Run the CLI in a scratch copy of tests/golden/data; returns (CompletedProcess, hits from
    KEYFOUNDKEYFOUND.txt / VANITYKEYFOUND.txt).  kill_after: stop it with SIGTERM after that many
    seconds (exit 124, as `timeout` reports), for runs that never end by themselves."""
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        cmd = [CLI] + argv + ["-q", "-s", "0"]
        if kill_after:
            cmd = ["timeout", "-k", "10", str(kill_after)] + cmd
        p = subprocess.run(cmd, cwd=td, capture_output=True, text=True, timeout=timeout)
        text = ""
        for fn in ("KEYFOUNDKEYFOUND.txt", "VANITYKEYFOUND.txt"):
            kf = os.path.join(td, fn)
            text += open(kf).read() if os.path.exists(kf) else ""
        p.hits_in_order = parse_keyfound(text, ordered=True)
        return p, parse_keyfound(text)


def without_threads(argv: list[str]) -> list[str]:
    """argv without its "-t N" pair (the engine's CLI takes -g for devices; other "8"s stay)."""
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == "-t" and i + 1 < len(argv):
            skip = True
            continue
        out.append(a)
    return out


def _uniq(xs):
    return [x for i, x in enumerate(xs) if x not in xs[:i]]


def check_against_reference(ref: dict, argv: list[str], name: str):
    """Run `argv` and compare exit status, KEYFOUND records and stdout hit blocks with the fixture.
    BSGS fixtures compare each distinct hit once: overlapping bases let several reference threads
    print the same key before the exit.  Fixtures of runs stopped after `killed_after` seconds
    compare the hits below `cmp_below` (the reference's threads covered those keys in time)."""
    kill = 8 if ref.get("killed_after") else None
    p, hits = run_cli(argv, kill_after=kill)
    assert p.returncode == ref["exit"], p.stdout[-2000:] + p.stderr[-2000:]
    blocks = sorted(STDOUT_BLOCK.findall(p.stdout))
    if "cmp_below" in ref:
        lim = int(ref["cmp_below"], 16)
        hits = [h for h in hits if int(h["key"], 16) < lim]
        blocks = [b for b in blocks if int(re.search(r"Key: ([0-9a-f]+)", b).group(1), 16) < lim]
    ref_hits, ref_blocks = ref["hits"], ref["stdout_blocks"]
    if name.startswith("bsgs"):
        hits, ref_hits, blocks, ref_blocks = _uniq(hits), _uniq(ref_hits), _uniq(blocks), _uniq(ref_blocks)
    assert hits == ref_hits
    if ref.get("killed_after"):
        # the stopped reference lost the tail of its block-buffered stdout: what it printed is there
        rest = list(blocks)
        for b in ref_blocks:
            assert b in rest, b
            rest.remove(b)
    else:
        assert blocks == ref_blocks
    if "hits_in_order" in ref:  # single-thread fixtures: the records in the reference's print order
        assert p.hits_in_order == ref["hits_in_order"]
    if "stderr_lines" in ref:  # the reference's notes on target-file lines it skipped, in order
        assert STDERR_NOTE.findall(p.stderr) == ref["stderr_lines"]
    if "stdout_notes" in ref:  # and on public keys it refused
        assert STDOUT_NOTE.findall(p.stdout) == ref["stdout_notes"]
    return p
