"""--mapped bloom files (keyhunt.cpp:724-806, 1131-1172, 1700-1785, 7630-7706; bloom/bloom.cpp:491-747)
against the reference CLI: each sequence of tests/golden/ref_mapped.json (oracle/make_golden.py
--mapped) is replayed with the engine's CLI in one scratch directory, and after every run the mapped
files are byte-identical to the ones the reference left -- a fresh filter, a reload (bits = bytes*8,
hash count from the file size, the items added again on top), chunked files, size overrides applied
to the first filter only, --create-mapped + --load-bloom, and the 768 BSGS shard files -- and the
hits are the reference's."""
import hashlib
import json
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from conftest import DATA, GOLDEN
from _cli import CLI, parse_keyfound

pytestmark = pytest.mark.gpu
REF = json.load(open(os.path.join(GOLDEN, "ref_mapped.json")))
SEQS = [k for k in REF if not k.startswith("_")]


def mapped_files(d: str) -> dict:
    out, layers = {}, {}
    for f in sorted(os.listdir(d)):
        m = re.match(r"(bloom2?3?-)(\d+)\.dat$", f)
        if m:
            layers.setdefault(m.group(1), {})[int(m.group(2))] = f
        elif f.startswith("data_") and f.endswith(".dat"):  # -S target cache: the mmap pointer masked
            b = bytearray(open(os.path.join(d, f), "rb").read())
            size = len(b)             # (masking a short file pads it, as the generator's digest does)
            b[96:104] = bytes(8)
            out[f] = [size, hashlib.sha256(bytes(b)).hexdigest()]
        elif f.startswith("keyhunt_bsgs_"):  # -S table files: each shard's struct bloom bf pointer masked
            b = bytearray(open(os.path.join(d, f), "rb").read())
            if f.endswith(".blm"):
                rec = len(b) // 256
                for i in range(256):
                    b[i * rec + 64: i * rec + 72] = bytes(8)
            out[f] = [len(b), hashlib.sha256(bytes(b)).hexdigest()]
        elif f.endswith(".dat") or re.search(r"\.dat\.\d+$", f):
            b = open(os.path.join(d, f), "rb").read()
            out[f] = [len(b), hashlib.sha256(b).hexdigest()]
    for pfx, shards in layers.items():
        h = hashlib.sha256()
        sizes = []
        for i in range(256):
            b = open(os.path.join(d, shards[i]), "rb").read()
            sizes.append(len(b))
            h.update(b)
        out[pfx + "*"] = [sizes, h.hexdigest()]
    return out


@pytest.mark.parametrize("name", SEQS)
def test_mapped_sequence_matches_reference(name):
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        for k, step in enumerate(REF[name]):
            argv = list(step["argv"])
            if "-t" in argv:  # the reference ran with -t 4; the engine's CLI takes -g contexts
                i = argv.index("-t")
                del argv[i:i + 2]
            p = subprocess.run([CLI] + argv + ["-q", "-s", "0"], cwd=td, capture_output=True, text=True, timeout=600)
            text = ""
            for fn in ("KEYFOUNDKEYFOUND.txt", "VANITYKEYFOUND.txt"):
                if os.path.exists(os.path.join(td, fn)):
                    text += open(os.path.join(td, fn)).read()
                    os.remove(os.path.join(td, fn))
            if step["exit"] < 0:  # the reference died of a signal (-S --mapped-chunks N>1): an error status here
                assert p.returncode > 0 and "[E]" in p.stderr, (k, p.returncode, p.stderr[-1500:])
            else:
                assert p.returncode == step["exit"], (k, p.stdout[-1500:], p.stderr[-1500:])
            if step.get("stderr_E") and step["exit"] > 0:
                assert [ln for ln in p.stderr.splitlines() if ln.startswith("[E]")] == step["stderr_E"], k
            hits, ref_hits = parse_keyfound(text), step["hits"]
            if "bsgs" in argv:  # several reference threads may print the key before the exit
                hits = [h for i, h in enumerate(hits) if h not in hits[:i]]
                ref_hits = [h for i, h in enumerate(ref_hits) if h not in ref_hits[:i]]
            assert hits == ref_hits, k
            assert mapped_files(td) == step["files"], k
