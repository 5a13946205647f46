"""The reference-side binding of INTEGRATION.md sections 2-3, compiled: integration/patch_reference.py
inserts the engine calls into a scratch copy of the reference's keyhunt.cpp and links it with the
reference's own objects and libkh_gpu.so (oracle/_ref/keyhunt_gpu, built by __graft_entry__.build()
in the development container and shipped with the tree).  With KH_GPU=1 its thread_process /
thread_process_bsgs hand every chunk / batch of bases to the engine, and the reference's own
writekey and BSGS hit printing report the keys: the KEYFOUNDKEYFOUND.txt records and stdout hit
blocks equal those of the unpatched reference CLI on the same arguments (tests/golden/ref_e2e.json)."""
import json
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from conftest import DATA, GOLDEN, REPO
from _cli import STDOUT_BLOCK, parse_keyfound

pytestmark = pytest.mark.gpu
E2E = json.load(open(os.path.join(GOLDEN, "ref_e2e.json")))
PATCHED = os.path.join(REPO, "oracle", "_ref", "keyhunt_gpu")
CASES = ["rmd160_66_window", "bsgs_125_window", "xpoint_63_window", "address_66_window", "bsgs_120_window",
         "rmd160_1to32_compress_2p20", "bsgs_test120_b120"]


@pytest.mark.parametrize("name", CASES)
def test_patched_reference_on_gpu_matches_reference(name):
    if not os.path.exists(PATCHED):
        pytest.fail("oracle/_ref/keyhunt_gpu missing: run integration/patch_reference.py (build() does)")
    ref = E2E[name]
    argv = [a for a in ref["argv"] if a not in ("-t", "8")] + ["-t", "1", "-q"]
    with tempfile.TemporaryDirectory() as td:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        p = subprocess.run([PATCHED] + argv, cwd=td, capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, KH_GPU="1"))
        text = open(os.path.join(td, "KEYFOUNDKEYFOUND.txt")).read() if os.path.exists(
            os.path.join(td, "KEYFOUNDKEYFOUND.txt")) else ""
    assert p.returncode == ref["exit"], p.stdout[-2000:] + p.stderr[-2000:]
    assert "kh_" not in p.stderr, p.stderr  # no engine error
    uniq = (lambda xs: [x for i, x in enumerate(xs) if x not in xs[:i]]) if name.startswith("bsgs") else (lambda xs: xs)
    assert uniq(parse_keyfound(text)) == uniq(ref["hits"])
    assert uniq(sorted(STDOUT_BLOCK.findall(p.stdout))) == uniq(ref["stdout_blocks"])
