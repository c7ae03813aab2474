#!/usr/bin/env python3
"""Per-kernel split of the C3 best-score table build (ulg_search_from_scores)
against its wall time, after one warm-up build."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

n, N, k = 25, 10000, 6
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
ctx.search_from_scores()
walls = []
for _ in range(3):
    t0 = time.perf_counter()
    ctx.search_from_scores()
    walls.append(1e3 * (time.perf_counter() - t0))
ctx.profile(True)
ctx.profile_select(None)
ctx.profile_reset()
t0 = time.perf_counter()
ctx.search_from_scores()
prof_wall = 1e3 * (time.perf_counter() - t0)
kern = ctx.profile_dump()
ctx.profile(False)
print(json.dumps({"wall_ms": walls, "profiled_wall_ms": prof_wall,
                  "kernels_ms": {kk: round(v["total_ms"], 4) for kk, v in kern.items()},
                  "kernel_sum_ms": sum(v["total_ms"] for v in kern.values())}))
ctx.close()
