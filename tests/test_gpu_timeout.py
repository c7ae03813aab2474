"""The reference's -r running-time budgets on the HIP path.

score: ScoreCalculator stops when its timer fires (score_calculator.cpp:
33-52,78,91) and keeps what it stored so far.  The GPU scores every variable
at once, layer by layer, and checks the budget after each complete layer
(ulg_set_option "time_limit_ms"), so whatever layer it stops after, the sets
it kept are exactly the full run's sets of at most that many parents (a
layer's decisions read only lower layers).
astar: the watchdog ends the search loop without a goal (astar_main.cpp:
135-138,266,535-540)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG
import synth

pytestmark = pytest.mark.gpu


def test_scorer_budget_keeps_whole_layers(ulg_ctx):
    n, N, k = 25, 10000, 6
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.set_option("time_limit_ms", 0)
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), full, k)
    assert ulg_ctx.info("out_of_time") == 0 and ulg_ctx.info("highest_completed_layer") == k
    try:
        ulg_ctx.set_option("time_limit_ms", 1)
        o2, s2, c2 = ulg_ctx.score_all(list(range(n)), full, k)
        done = ulg_ctx.info("highest_completed_layer")
        assert ulg_ctx.info("out_of_time") == (1 if done < k else 0)
    finally:
        ulg_ctx.set_option("time_limit_ms", 0)
    assert 1 <= done <= k
    for v in range(n):
        a, fa = sets[offs[v]:offs[v + 1]], scores[offs[v]:offs[v + 1]]
        keep = np.array([bin(int(x)).count("1") <= done for x in a], dtype=bool)
        assert np.array_equal(s2[o2[v]:o2[v + 1]], a[keep]), v
        assert c2[o2[v]:o2[v + 1]].tobytes() == fa[keep].tobytes(), v


def test_exact_astar_watchdog(ulg_ctx, tmp_path):
    """C3's exact-order search takes ~30 s; a 1 ms budget ends it without a
    goal, and the CLI prints the reference's messages and writes no netFile."""
    n, N, k = 25, 10000, 6
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), full, k)
    ulg_ctx.search_from_scores()
    try:
        ulg_ctx.set_option("time_limit_ms", 1)
        res = ulg_ctx.astar(edges=full, mode=0, net_text=True)
        assert ulg_ctx.info("out_of_time") == 1
        assert res["net_text"] == ""
        assert res["expanded"] < 26117314  # the watchdog may fire before the first pop
    finally:
        ulg_ctx.set_option("time_limit_ms", 0)
    data = tmp_path / "c3.csv"
    synth.write_csv(str(data), X)
    pss = tmp_path / "c3.pss"
    r = subprocess.run([os.path.join(PKG, "bin", "score"), str(data), str(pss), "-f", "cBIC", "--lambda", "2",
                        "-p", str(k)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    net = tmp_path / "net"
    r = subprocess.run([os.path.join(PKG, "bin", "astar"), str(pss), "-n", str(net), "-r", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Maximum running time: 1" in r.stdout
    assert "Out of time" in r.stdout and "No solution found." in r.stdout
    assert not net.exists()

