"""Times the best-score table build at C3 (per-kernel HIP events, repeat builds)."""
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
ctx.search_from_scores()  # allocations
ctx.profile(True)
ctx.profile_reset()
walls = []
for _ in range(5):
    t = time.perf_counter()
    ctx.search_from_scores()
    walls.append(1e3 * (time.perf_counter() - t))
d = ctx.profile_dump()
print("wall ms", [round(w, 2) for w in walls])
for name, v in sorted(d.items()):
    if name.startswith("bs_") or name.startswith("quantize"):
        print(name, v["count"], round(v["total_ms"] / max(v["count"], 1), 3), "ms avg")
