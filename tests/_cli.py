"""Helpers to run the engine's CLI (keyhunt_amd/bin/keyhunt-amd) like the reference binary."""
import os
import re
import shutil
import subprocess
import tempfile

from conftest import DATA, REPO

CLI = os.path.join(REPO, "keyhunt_amd", "bin", "keyhunt-amd")


def parse_keyfound(text: str) -> list[dict]:
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
    return sorted(hits, key=lambda h: int(h["key"], 16))


def run_cli(argv: list[str], timeout: int = 600):
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        p = subprocess.run([CLI] + argv + ["-q", "-s", "0"], cwd=td, capture_output=True, text=True, timeout=timeout)
        text = ""
        for fn in ("KEYFOUNDKEYFOUND.txt", "VANITYKEYFOUND.txt"):
            kf = os.path.join(td, fn)
            text += open(kf).read() if os.path.exists(kf) else ""
        return p, parse_keyfound(text)
