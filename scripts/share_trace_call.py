#!/usr/bin/env python3
"""One rank's 8-way share of C3 (shard.assign), scored alone on one GPU:
warm calls, for a rocprofv3 kernel trace of a single call's timeline
(scripts/trace_timeline.py prints it).

    python scripts/share_trace_call.py [--ranks 8] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
n, N, k = 25, 10000, 6
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
cands = [(1 << n) - 1] * n
parts = shard.assign(n, a.ranks, cands, k)
p = max(parts, key=len)
for _ in range(a.reps):
    ctx.score(list(p), [cands[v] for v in p], k)
print("variables", list(p))
ctx.close()
