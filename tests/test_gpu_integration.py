"""The reference-side binding of INTEGRATION.md sections 1-3, compiled: integration/patch_reference.py
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
import time

import pytest

from conftest import DATA, GOLDEN, REPO
from _cli import STDOUT_BLOCK, parse_keyfound, without_threads

pytestmark = pytest.mark.gpu
E2E = json.load(open(os.path.join(GOLDEN, "ref_e2e.json")))
PATCHED = os.path.join(REPO, "oracle", "_ref", "keyhunt_gpu")
CASES = ["rmd160_66_window", "bsgs_125_window", "xpoint_63_window", "address_66_window", "bsgs_120_window",
         "rmd160_1to32_compress_2p20", "bsgs_test120_b120",
         # --rmd-batch-size below 1024: the binding hands the reference's group size to kh_set_rmd_batch
         "rmd160_batch512_both", "rmd160_batch1001_compress_endo"]


def run_patched(argv, td=None, timeout=600):
    """(process, KEYFOUNDKEYFOUND.txt text, wall seconds) of the patched reference with KH_GPU=1, run
    in `td` (a fresh directory holding the fixture inputs when None)."""
    if not os.path.exists(PATCHED):
        pytest.fail("oracle/_ref/keyhunt_gpu missing: run integration/patch_reference.py (build() does)")
    own = td is None
    if own:
        td = tempfile.mkdtemp()
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
    try:
        t0 = time.time()
        p = subprocess.run([PATCHED] + argv, cwd=td, capture_output=True, text=True, timeout=timeout,
                           env=dict(os.environ, KH_GPU="1"))
        wall = time.time() - t0
        kf = os.path.join(td, "KEYFOUNDKEYFOUND.txt")
        text = open(kf).read() if os.path.exists(kf) else ""
    finally:
        if own:
            shutil.rmtree(td, ignore_errors=True)
    return p, text, wall


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("threads", [1, 2])
def test_patched_reference_on_gpu_matches_reference(name, threads):
    """-t 1 and -t 2: with two threads both workers share the device's one context (section 1)."""
    ref = E2E[name]
    argv = without_threads(ref["argv"]) + ["-t", str(threads), "-q"]
    p, text, _ = run_patched(argv)
    assert p.returncode == ref["exit"], p.stdout[-2000:] + p.stderr[-2000:]
    assert "kh_" not in p.stderr, p.stderr  # no engine error
    uniq = (lambda xs: [x for i, x in enumerate(xs) if x not in xs[:i]]) if name.startswith("bsgs") else (lambda xs: xs)
    assert uniq(parse_keyfound(text)) == uniq(ref["hits"])
    assert uniq(sorted(STDOUT_BLOCK.findall(p.stdout))) == uniq(ref["stdout_blocks"])


def test_patched_reference_bench_geometry_k128_without_cpu_tables():
    """configs[3] geometry (-k 128: M = 2^29 baby steps) on puzzle 125's known-answer window: the
    patched reference takes its tables from the engine (kh_bsgs_build on the GPU, no thread_bPload
    pool: ~120 s on 8 cores and 1.9 GB of host blooms in the unpatched reference) and finds the key
    in well under 15 s."""
    ref = E2E["bsgs_125_window"]
    argv = without_threads(ref["argv"]) + ["-k", "128", "-t", "1"]
    p, text, wall = run_patched(argv)
    assert p.returncode == 1, p.stdout[-2000:] + p.stderr[-2000:]
    assert parse_keyfound(text) == ref["hits"]
    assert "MI355X engine: bloom filters and bP table for 536870912 baby steps built on 1 GPU(s)" in p.stdout
    assert "processing" not in p.stdout and "Bloom filter for" not in p.stdout  # no CPU baby-step build
    assert wall < 15, wall


def test_patched_reference_bsgs_table_files():
    """-S: the first run builds the tables on the GPU and writes the reference's four files
    (kh_bsgs_save); the second reads them back (kh_bsgs_load) and finds the same key; the
    unpatched reference reads the engine's files too (tests/test_gpu_tables.py)."""
    ref = E2E["bsgs_120_window"]
    argv = without_threads(ref["argv"]) + ["-t", "1", "-S"]
    td = tempfile.mkdtemp()
    try:
        for fn in os.listdir(DATA):
            shutil.copy(os.path.join(DATA, fn), td)
        p1, t1, _ = run_patched(argv, td)
        files = sorted(f for f in os.listdir(td) if f.startswith("keyhunt_bsgs_"))
        os.remove(os.path.join(td, "KEYFOUNDKEYFOUND.txt"))
        p2, t2, _ = run_patched(argv, td)
    finally:
        shutil.rmtree(td, ignore_errors=True)
    assert p1.returncode == 1 and p2.returncode == 1, p1.stdout[-1500:] + p2.stdout[-1500:] + p2.stderr[-1500:]
    assert "built on 1 GPU(s)" in p1.stdout and "read from the -S files on 1 GPU(s)" in p2.stdout
    assert [f.split("_")[2] for f in files] == ["2", "4", "6", "7"]
    assert parse_keyfound(t1) == parse_keyfound(t2) == ref["hits"]
