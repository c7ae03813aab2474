#!/usr/bin/env python3
"""One rank's C3 share (shard.assign over --ranks, --rank) scored repeatedly:
run under rocprofv3 --kernel-trace to see the call's kernel timeline (the
strong-scaling floor is the chain of dependent launches, not the work)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--calls", type=int, default=30)
a = ap.parse_args()
n, N, k = 25, 10000, 6
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
cands = [(1 << n) - 1] * n
part = list(shard.assign(n, a.ranks, cands, k)[a.rank]) if a.ranks > 1 else list(range(n))
ts = []
for _ in range(a.calls):
    t = time.perf_counter()
    ctx.score(part, [cands[v] for v in part], k)
    ts.append(time.perf_counter() - t)
print("variables", part, "best ms %.4f median ms %.4f" % (min(ts) * 1e3, sorted(ts)[len(ts) // 2] * 1e3), flush=True)
ctx.close()
