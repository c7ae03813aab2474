"""When walk_sliced may insert an expanded node into `checked` (round 6).

scripts/walk_mark_order_check.cpp replays find_best_subset_score
(BIC_OLS.cpp:125-172) on random present / hi bitsets, layers 2..8, both
phases, with the reference's insert order and with the forms walk_sliced
uses: the flattened second-deepest level (its callees only test; one insert
at the end, only when a call ran) must decide every set as the reference
does.  Inserting before the calls is the counter-example: it must differ
somewhere, or the check has lost its power.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "scripts", "walk_mark_order_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_walk_insert_forms_decide_as_the_reference(tmp_path):
    exe = tmp_path / "walk_mark_order_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), SRC], check=True)
    out = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    m = re.search(r"first call only (\d+), before the calls (\d+), flat second-deepest level (\d+)", out.stdout)
    assert m, out.stdout + out.stderr
    first, before, flat = (int(x) for x in m.groups())
    assert first == 0 and flat == 0, out.stdout
    assert before > 0, out.stdout
    assert out.returncode == 0
