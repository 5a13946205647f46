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

import pytest

from conftest import GOLDEN
from _cli import check_against_reference, without_threads

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
