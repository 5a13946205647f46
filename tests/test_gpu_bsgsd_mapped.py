"""bsgsd-amd's bloom-file options against the reference daemon's own starts
(tests/golden/ref_bsgsd_mapped.json, oracle/make_golden.py --bsgsd-mapped).

Each case is a sequence of daemon starts in one directory (bsgsd.cpp:776-889 options,
584-660 initBloomFilterMapped, 955-995 --create-mapped, 1180-1255 the shard filters): whether the
start came up, its exit status when it did not, the [E]/[W] lines, the reply to one found request,
and every file left behind -- the 3 x 256 shard files (per layer and chunk: sizes and the sha256 of
their concatenation), the -S files (masked digests) and the --create-mapped file -- must equal the
reference's.  Covered: --mapped fresh and reloaded (the reload re-inserts with the geometry
bloom_load_mmap derives from the file size), --load-bloom with and without the files,
--mapped=NAME with --mapped-chunks, the size overrides (--mapped-size, --bloom-bytes,
--create-mapped=N: bsgsd's sizing picks 2^62 entries for any size, so those starts fail as the
reference's do), --create-mapped without a size, a plain start over shard files, and
--bsgs-block-count/--bsgs-block-size/--tmpdir/--rmd-batch-size (no effect on the daemon)."""
import json
import os
import re
import socket
import subprocess
import sys
import time

import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "oracle"))
import make_golden  # noqa: E402  (test infrastructure: the fixture's own file digests)

pytestmark = pytest.mark.gpu
DAEMON = os.path.join(REPO, "keyhunt_amd", "bin", "bsgsd-amd")
REF = json.load(open(os.path.join(GOLDEN, "ref_bsgsd_mapped.json")))
CASES = [k for k in REF if not k.startswith("_") and k not in ("args", "request")]


def _start(cwd, logp, extra):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    log = open(logp, "w")
    p = subprocess.Popen([DAEMON] + REF["args"] + ["-g", "1"] + extra + ["-p", str(port), "-i", "127.0.0.1"],
                         cwd=cwd, stdout=log, stderr=subprocess.STDOUT)
    t0 = time.time()
    while p.poll() is None and "Listening in" not in open(logp).read():
        assert time.time() - t0 < 150, "bsgsd-amd neither listened nor exited"
        time.sleep(0.2)
    step = {"listened": p.poll() is None}
    if step["listened"]:
        with socket.create_connection(("127.0.0.1", port), timeout=120) as c:
            c.sendall(REF["request"].encode())
            reply = b""
            while True:
                b = c.recv(4096)
                if not b:
                    break
                reply += b
        step["reply"] = reply.decode()
        p.kill()
    p.wait(timeout=60)
    log.close()
    if not step["listened"]:
        step["exit"] = p.returncode
    return step


@pytest.mark.parametrize("name", CASES)
def test_bsgsd_mapped_options_match_reference(tmp_path, name):
    d = tmp_path / "run"
    d.mkdir()
    (d / "tmpdir_x").mkdir()
    logp = str(tmp_path / "daemon.log")
    for i, ref in enumerate(REF[name]):
        got = _start(str(d), logp, ref["extra"])
        text = open(logp).read()
        kf = d / "KEYFOUNDKEYFOUND.txt"
        if kf.exists():
            kf.unlink()
        where = f"{name} start {i} {ref['extra']}"
        assert got["listened"] == ref["listened"], (where, text[-2000:])
        if ref["listened"]:
            assert got["reply"] == ref["reply"], where
        else:
            assert got["exit"] == ref["exit"], (where, text[-2000:])
        notes = sorted(set(m.strip() for m in re.findall(r"\[[EW]\] [^\n]*", text)))
        assert notes == ref["notes"], where
        assert make_golden.bsgsd_dir_files(str(d)) == ref["files"], where
        assert sorted(os.listdir(d / "tmpdir_x")) == ref["tmpdir_files"], where
