"""Per-kernel times (HIP events, one profiled C3 scoring call after warm-up):
the A/B companion of score_time.py for alternative builds (ULG_LIB=path)."""
import os
import sys

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
    ctx.score(list(range(n)), full, k)
ctx.profile(True)
ctx.profile_select(None)
ctx.profile_reset()
ctx.score(list(range(n)), full, k)
kern = ctx.profile_dump()
ctx.profile(False)
keys = ["score_layer_5_rest", "walk_5_rest", "score_layer_6_var0", "walk_6_var0", "score_layer_6_rest", "walk_6_rest"]
print(os.environ.get("ULG_LIB", "default").split("/")[-2], " ".join(f"{kk}={kern[kk]['total_ms']:.4f}" for kk in keys if kk in kern),
      flush=True)
