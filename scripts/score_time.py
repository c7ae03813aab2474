"""Wall time of back-to-back C3 scoring calls (no profiling): the A/B driver
for alternative builds of libulg.so (ULG_LIB=path)."""
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
full = [(1 << n) - 1] * n
for _ in range(5):
    stored, scored = ctx.score(list(range(n)), full, k)
best = 1e9
for rep in range(3):
    t = time.perf_counter()
    K = 100
    for _ in range(K):
        ctx.score(list(range(n)), full, k)
    best = min(best, (time.perf_counter() - t) / K)
print(f"{os.environ.get('ULG_LIB', 'default')} c3 {best * 1e3:.4f} ms per call, {stored} of {scored} stored",
      flush=True)
