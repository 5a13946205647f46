"""The address family's mapped bloom files and -S data files, on the CPU.

keyhunt-amd creates, reloads and fills a --mapped target filter (keyhunt.cpp:7630-7706) and, with -S,
writes the data_<hex>.dat cache (writeFileIfNeeded, 7756-7855) before it looks for a device: the
filter gates exact checks only, so its bits come from the target rows on the host.  Run here without a
GPU, each address-family sequence of tests/golden/ref_mapped.json (oracle/make_golden.py --mapped,
the reference CLI's runs) leaves byte-identical files after every step; the hits are compared on the
GPU (tests/test_gpu_mapped.py).  BSGS shard files are filled by the GPU's baby steps and are only
checked there."""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

from conftest import DATA, GOLDEN
from _cli import CLI
from test_gpu_mapped import mapped_files

REF = json.load(open(os.path.join(GOLDEN, "ref_mapped.json")))
SEQS = [k for k in REF if not k.startswith("_") and not any("bsgs" in s["argv"] for s in REF[k])]


@pytest.mark.parametrize("name", SEQS)
def test_address_family_mapped_files_match_reference(name):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        for k, step in enumerate(REF[name]):
            argv = list(step["argv"])
            if "-t" in argv:
                i = argv.index("-t")
                del argv[i:i + 2]
            p = subprocess.run([CLI] + argv + ["-q", "-s", "0"], cwd=td, capture_output=True, text=True, timeout=120,
                               env=env)
            assert mapped_files(td) == step["files"], (k, step["argv"])
            if step["exit"] < 0:       # the reference died of a signal (-S --mapped-chunks N>1): an error here
                assert p.returncode != 0 and "[E]" in p.stderr, (k, p.returncode, p.stderr)
            elif step.get("stderr_E"):  # a clean failure before any device work: the same [E] lines and status
                assert p.returncode == step["exit"], (k, p.returncode, p.stderr)
                assert [ln for ln in p.stderr.splitlines() if ln.startswith("[E]")] == step["stderr_E"]
