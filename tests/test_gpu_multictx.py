"""Several engine contexts sharing the reference's work cursor (keyhunt.cpp:2717-2839 thread spawn,
3321-3324 chunk cursor, 4600-4617 base cursor): every reference-CLI fixture of
tests/golden/ref_e2e.json run with `-g 2` and `-g 3` on one device gives the reference's hit set.

The contexts are opened on devices d % ndev, so on a one-GPU box they share it, each with its own
tables, lanes and host thread, exactly as on an 8-GPU node each takes its own device.  The window
fixtures hold 4 to 16 chunks of 2^20 keys (`-n` cannot go below 2^20, validate_nk) or several BSGS
bases, so the contexts really split them; the 2^20-key ones are one chunk, taken by one context while
the others find the cursor at its end."""
import json
import os
import re

import pytest

from conftest import GOLDEN
from _cli import check_against_reference, run_cli, without_threads

pytestmark = pytest.mark.gpu
E2E = json.load(open(os.path.join(GOLDEN, "ref_e2e.json")))
CASES = [k for k in E2E if not k.startswith("_")]


def _argv(name: str, contexts: int) -> list[str]:
    return without_threads(E2E[name]["argv"]) + ["-g", str(contexts)]


@pytest.mark.parametrize("contexts", [2, 3])
@pytest.mark.parametrize("name", CASES)
def test_cli_contexts_match_reference(name, contexts):
    p = check_against_reference(E2E[name], _argv(name, contexts), name)
    if E2E[name]["exit"] != 255:  # the run got as far as opening its contexts (not a refused target file)
        assert f"({contexts} contexts)" in p.stdout


def test_cli_refuses_contexts_beyond_device_memory():
    """-g contexts stacked on one device must fit its free memory: at the default
    2^32-key chunk each rmd160 context holds a 64 GB inversion pad (kh_scan_memory), so -g 8 on one
    288 GB GPU is refused before any context opens, with the figures; xpoint's sparse pad is half."""
    import ctypes
    from keyhunt_amd.engine import lib
    need = ctypes.c_uint64(0)
    assert lib().kh_scan_memory(ctypes.c_uint64(1 << 32), 0, 0, ctypes.byref(need)) == 0
    assert need.value >= 64 << 30
    xp = ctypes.c_uint64(0)
    assert lib().kh_scan_memory(ctypes.c_uint64(1 << 32), 1, 0, ctypes.byref(xp)) == 0
    assert 32 << 30 <= xp.value < need.value
    p, hits = run_cli(["-m", "rmd160", "-f", "66.rmd", "-l", "compress", "-b", "66", "-g", "8"], timeout=120)
    assert p.returncode == 1, p.stderr[-2000:]
    assert re.search(r"-g 8: 8 context\(s\) on GPU 0 need [\d.]+ GB of device memory \([\d.]+ GB each\)", p.stderr), p.stderr
    assert not hits
