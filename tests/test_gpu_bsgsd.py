"""bsgsd-amd: the reference's BSGS daemon protocol (bsgsd.cpp:3307-3579, BSGSD.md) on the GPU
engine.  One request per connection, line mode and HTTP POST/JSON mode, replies as the reference
sends them; tables written as -S files on first start and read back on the next."""
import http.client
import json
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
    def __init__(self, cwd, n="0x1000000", k="2"):
        self.port = free_port()
        self.log = open(os.path.join(cwd, "bsgsd.log"), "w+")
        self.p = subprocess.Popen([DAEMON, "-n", n, "-k", k, "-g", "1", "-p", str(self.port), "-i", "127.0.0.1"], cwd=cwd,
                                  stdout=self.log, stderr=subprocess.STDOUT)
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


def test_line_and_http_protocol(workdir):
    d = Daemon(str(workdir))
    try:
        # found (puzzle 63's key), both request spellings of the range
        assert d.line(f"{PUB63} 7cce5efdac000000:7cce5efdad000000\n".encode()) == (KEY63 + "\n").encode()
        assert d.line(f"{PUB63} 7cce5efdac000000 7cce5efdad000000\n".encode()) == (KEY63 + "\n").encode()
        # not in range
        assert d.line(f"{PUB63} 4000000000000000:4000000001000000\n".encode()) == b"404 Not Found\n"
        # bad requests (bsgsd.cpp:3440-3490)
        assert d.line(b"nonsense\n") == b"400 Bad Request"
        assert d.line(f"{PUB63} 7cce5efdac000000\n".encode()) == b"400 Bad Request"
        assert d.line(f"{PUB63} zz:7cce5efdad000000\n".encode()) == b"400 Bad Request"
        assert d.line(b"0465ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579 1:2\n") == b"400 Bad Request"
        # HTTP POST / JSON
        c = http.client.HTTPConnection("127.0.0.1", d.port, timeout=120)
        c.request("POST", "/", body=json.dumps({"pubkey": PUB63, "from": "7cce5efdac000000", "to": "7cce5efdad000000"}),
                  headers={"Content-Type": "application/json"})
        r = c.getresponse()
        assert (r.status, r.read()) == (200, (KEY63 + "\n").encode())
        assert r.getheader("Content-Type") == "text/plain" and float(r.getheader("X-Elapsed-Seconds")) >= 0
        c = http.client.HTTPConnection("127.0.0.1", d.port, timeout=120)
        c.request("POST", "/", body=json.dumps({"pubkey": PUB63, "from": "4000000000000000", "to": "4000000001000000"}))
        r = c.getresponse()
        assert (r.status, r.read()) == (404, b"404 Not Found\n")
        c = http.client.HTTPConnection("127.0.0.1", d.port, timeout=120)
        c.request("POST", "/", body=json.dumps({"pubkey": PUB63}))
        assert c.getresponse().status == 400
        kf = open(workdir / "KEYFOUNDKEYFOUND.txt").read()
        assert kf.count(f"Key found privkey {KEY63}\nPublickey {PUB63}\n") == 3
    finally:
        d.stop()


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
