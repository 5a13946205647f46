"""bsgsd-amd --create-mapped on the CPU (it exits before touching a GPU, bsgsd.cpp:955-995): the
exit status, [E] lines and files of the reference daemon's own runs (tests/golden/ref_bsgsd_mapped.json;
the full start sequences run in tests/test_gpu_bsgsd_mapped.py)."""
import json
import os
import re
import subprocess
import sys

import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "oracle"))
import make_golden  # noqa: E402

DAEMON = os.path.join(REPO, "keyhunt_amd", "bin", "bsgsd-amd")
REF = json.load(open(os.path.join(GOLDEN, "ref_bsgsd_mapped.json")))
STEPS = [(name, i) for name in REF if not name.startswith("_") and name not in ("args", "request")
         for i, st in enumerate(REF[name]) if any(a.startswith("--create-mapped") for a in st["extra"])]


@pytest.mark.skipif(not os.path.exists(DAEMON), reason="bsgsd-amd not built")
@pytest.mark.parametrize("name,i", STEPS)
def test_create_mapped_matches_reference(tmp_path, name, i):
    ref = REF[name][i]
    assert i == 0 and not ref["listened"]
    p = subprocess.run([DAEMON] + REF["args"] + ref["extra"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert p.returncode == ref["exit"]
    assert sorted(set(m.strip() for m in re.findall(r"\[[EW]\] [^\n]*", p.stdout + p.stderr))) == ref["notes"]
    assert make_golden.bsgsd_dir_files(str(tmp_path)) == ref["files"]
