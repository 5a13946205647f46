"""kh_cols.h is generated (tools/gen_cols.py): the committed header must be what the generator emits
now, and the generator's own hazard checker (every carry count >= 2 wait states after the
multiply-add that wrote its mask, no mask reused before it is read) must pass for every column shape
it schedules."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_kh_cols_header_is_generated():
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_cols.py")], check=True,
                         capture_output=True, text=True).stdout
    assert out == open(os.path.join(REPO, "keyhunt_amd", "csrc", "kh_cols.h")).read()


def test_column_schedules_respect_the_mask_hazard():
    import gen_cols as G
    for n in range(1, 9):
        for safe in range(0, n + 1):
            G.check(G.schedule(n, safe), n, safe)   # asserts inside
