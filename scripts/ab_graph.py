#!/usr/bin/env python3
"""A/B of the captured scoring graph (ulg_set_option score_graph): wall time
of K back-to-back scoring calls per config, no profiling, alternating."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

ctx = ulg.Context(0)
for name, (n, N, k) in {"c2": (20, 10000, 4), "c3": (25, 10000, 6)}.items():
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx.load(X, 2.0)
    full = [(1 << n) - 1] * n
    for rep in range(3):
        for g in (0, 1):
            ctx.set_option("score_graph", g)
            for _ in range(5):
                ctx.score(list(range(n)), full, k)
            t = time.perf_counter()
            K = 100
            for _ in range(K):
                ctx.score(list(range(n)), full, k)
            dt = (time.perf_counter() - t) / K
            print(f"{name} graph={g} {dt * 1e3:.4f} ms per call", flush=True)
