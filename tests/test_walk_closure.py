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


def test_cpp_walk_may_hit_equals_restatement():
    """The C++ walk_may_hit (csrc/cbic_dev.h, built for the host as
    bin/walk_may_hit_check from the same header the kernels include) reports
    exactly the testable set of scripts/walk_closure_check.py's restatement on
    random presence patterns of layers 1..6, both phases (the proof
    above checks the restatement; this pins the shipped function to it)."""
    import random
    pkg = os.path.join(ROOT, "urlearning-cpp_amd")
    subprocess.run(["make", "-C", pkg, "bin/walk_may_hit_check"], check=True, capture_output=True, timeout=600)
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import walk_closure_check as wc
    rng = random.Random(23)
    cases, lines = [], []
    for _ in range(3000):
        L, phase = rng.randint(1, 6), rng.randint(0, 1)
        Q = L if phase == 0 else L + 1
        W = wc.bits_words(L)
        pp = rng.random()
        pres = [0] * W
        for t in range(1 << Q):
            if rng.random() < pp:
                pres[t >> 6] |= 1 << (t & 63)
        cases.append((L, phase, pres))
        lines.append(f"{L} {phase} " + " ".join(f"{w:x}" for w in pres))
    r = subprocess.run([os.path.join(pkg, "bin", "walk_may_hit_check")], input="\n".join(lines) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.split("\n")
    for (L, phase, pres), got in zip(cases, out):
        W = wc.bits_words(L)
        _, tested = wc.walk_may_hit(L, phase, pres, [0] * W)
        assert [int(x, 16) for x in got.split()] == tested, (L, phase, pres)
