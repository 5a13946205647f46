"""bsgsd-amd: the reference's BSGS daemon (bsgsd.cpp:3307-3579, BSGSD.md) on the GPU engine, pinned
to a transcript of the reference daemon itself (tests/golden/ref_bsgsd.json): one request per
connection, line mode and HTTP POST/JSON mode, the same reply bytes and printed lines; the same
table files (-S, .tbl.md5, --ptable / --ptable-cache / --load-ptable) on start and restart."""
import json
import re
import os
import socket
import subprocess
import time

import pytest

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu
DAEMON = os.path.join(REPO, "keyhunt_amd", "bin", "bsgsd-amd")
PUB63 = "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579"
KEY63 = "7cce5efdaccf6808"
REF_TABLES = json.load(open(os.path.join(GOLDEN, "ref_tables.json")))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Daemon:
    def __init__(self, cwd, n="0x1000000", k="2", g="1", extra=()):
        self.port = free_port()
        self.log = open(os.path.join(cwd, "bsgsd.log"), "w+")
        self.p = subprocess.Popen([DAEMON, "-n", n, "-k", k, "-g", g, "-p", str(self.port), "-i", "127.0.0.1"] + list(extra),
                                  cwd=cwd, stdout=self.log, stderr=subprocess.STDOUT)
        t0 = time.time()
        while time.time() - t0 < 120:
            self.log.seek(0)
            if "Listening in" in self.log.read():
                return
            assert self.p.poll() is None, "daemon exited"
            time.sleep(0.2)
        raise TimeoutError("daemon did not start")

    def output(self):
        self.log.seek(0)
        return self.log.read()

    def line(self, msg: bytes, timeout=120) -> bytes:
        with socket.create_connection(("127.0.0.1", self.port), timeout=timeout) as s:
            s.sendall(msg)
            out = b""
            while True:
                b = s.recv(1024)
                if not b:
                    return out
                out += b

    def stop(self):
        self.p.kill()
        self.p.wait(timeout=30)
        self.text = self.output()
        self.log.close()


@pytest.fixture
def workdir(tmp_path):
    return tmp_path


REF_BSGSD = json.load(open(os.path.join(GOLDEN, "ref_bsgsd.json")))


def mask_elapsed(reply: bytes) -> bytes:
    import re
    return re.sub(rb"X-Elapsed-Seconds: [0-9.]+", b"X-Elapsed-Seconds: *", reply)


@pytest.mark.parametrize("contexts", ["1", "2"])
def test_transcript_matches_reference_daemon(workdir, contexts):
    """Every request of the reference daemon's transcript (tests/golden/ref_bsgsd.json, recorded from
    oracle/_ref/bsgsd built from bsgsd.cpp by oracle/Makefile.ref) gets the same reply bytes
    (X-Elapsed-Seconds masked) and the daemon prints the same lines for it; KEYFOUNDKEYFOUND.txt ends
    up identical.  With -g 2 two contexts share the GPU and split each request's bases."""
    d = Daemon(str(workdir), n=REF_BSGSD["args"][1], k=REF_BSGSD["args"][3], g=contexts)
    try:
        for i, r in enumerate(REF_BSGSD["requests"]):
            before = len(d.output())
            reply = d.line(r["request"].encode())
            t0 = time.time()
            while d.output().count("[+] Closing") < i + 1 and time.time() - t0 < 30:
                time.sleep(0.05)
            lines = [ln for ln in d.output()[before:].split("\n")
                     if ln and not ln.startswith(("[+] Accepting", "[+] Closing"))]
            assert mask_elapsed(reply).decode() == r["reply"], r["name"]
            assert lines == r["stdout"], r["name"]
        assert open(workdir / "KEYFOUNDKEYFOUND.txt").read() == REF_BSGSD["keyfound"]
    finally:
        d.stop()


def test_table_files_match_reference_daemon(tmp_path):
    """The reference daemon's start sequences (tests/golden/ref_bsgsd.json "starts"): the -S files
    plus keyhunt_bsgs_2_<M3>.tbl.md5, and with --ptable / --ptable-cache / --load-ptable the bP table
    file, its FILE.md5 and FILE.cache -- written from the rows the file held before the build, as the
    reference does -- are byte-identical (heap pointers masked), with the same bP-table messages."""
    from test_gpu_tables import masked_digest
    work = None
    for st in REF_BSGSD["starts"]:
        if st["fresh"]:
            work = tmp_path / st["name"]
            work.mkdir()
        d = Daemon(str(work), n=REF_BSGSD["args"][1], k=REF_BSGSD["args"][3], extra=st["extra"])
        d.stop()
        got = {f: masked_digest(str(work / f)) for f in sorted(os.listdir(work)) if f != "bsgsd.log"}
        assert got == st["files"], st["name"]
        assert [ln.strip() for ln in d.text.split("\n") if "bP table" in ln] == st["bptable_lines"], st["name"]


def test_tables_written_then_read(workdir):
    from test_gpu_tables import masked_digest
    d = Daemon(str(workdir))
    d.stop()
    for f, dig in REF_TABLES["n1000000_k2"]["files"].items():
        assert masked_digest(str(workdir / f)) == dig, f
    assert "Built 1 GPU table set" in d.text
    d = Daemon(str(workdir))
    try:
        assert "Read 1 GPU table set" in d.output()
        assert d.line(f"{PUB63} 7cce5efdac000000:7cce5efdad000000\n".encode()) == (KEY63 + "\n").encode()
    finally:
        d.stop()


def test_contexts_beyond_device_memory_are_refused(tmp_path):
    """-g stacks contexts on a device, each with its own tables and walk pad: a count that cannot
    fit the device's free memory is refused before any table is built (the old daemon ran
    out of memory after the first context's build)."""
    t0 = time.time()
    p = subprocess.run([DAEMON, "-n", "0x100000000000", "-k", "512", "-g", "64", "-p", str(free_port())],
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert re.search(r"-g 64: \d+ context\(s\) on GPU 0 need [\d.]+ GB of device memory", p.stderr), p.stderr
    assert not any(f.startswith("keyhunt_bsgs_") for f in os.listdir(tmp_path))  # nothing built or written
    assert time.time() - t0 < 120
