"""The two-pass scorer stores a queued set without its walk when no key
>= -ts lies among the nodes the walk can test (walk_may_hit, csrc/cbic_dev.h).
scripts/walk_closure_check.py restates that closure word by word and checks
it against find_best_subset_score's recursion (BIC_OLS.cpp:125-172 with the
reference's zero padding and `checked`, as walk_sliced replays it) on random
presence / hi patterns of layers 1..6, both phases: every node the recursion
tests is in the closure, so no walk that would prune a set is skipped."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_walk_closure_covers_the_recursion():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "walk_closure_check.py"), "--trials", "20000",
                        "--seed", "17"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "violations 0" in r.stdout
