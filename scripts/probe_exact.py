"""Times the exact-order A* (host replay over GPU tables) at C2 and C3."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

ctx = ulg.Context(0)
CFG = {"c2": (20, 10000, 4), "c3": (25, 10000, 6)}
for name in (sys.argv[1:] or ["c2", "c3"]):
    n, N, k = CFG[name]
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), full, k)
    ctx.search_from_scores()
    t = time.perf_counter()
    r = ctx.astar(edges=full, mode=0, net_text=False)
    dt = time.perf_counter() - t
    print(name, "exact A*:", r["expanded"], "expansions in %.3f s = %.3g /s" % (dt, r["expanded"] / dt),
          "cost", r["cost"], flush=True)
