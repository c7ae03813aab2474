"""Per-kernel time (HIP events) of one C3 scoring call, for A/B library
builds (ULG_LIB=...)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth, ulg
n, N, k = 25, 10000, 6
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
full = [(1 << n) - 1] * n
if len(sys.argv) > 1:
    ctx.set_option("score_variant", int(sys.argv[1]))
for _ in range(3):
    ctx.score(list(range(n)), full, k)
import time
t0 = time.perf_counter()
for _ in range(20):
    ctx.score(list(range(n)), full, k)
print(f"variant {sys.argv[1] if len(sys.argv) > 1 else 'default'}: {1e3 * (time.perf_counter() - t0) / 20:.3f} ms per call")
ctx.profile(True)
ctx.profile_reset()
for _ in range(10):
    ctx.score(list(range(n)), full, k)
d = ctx.profile_dump()
ctx.profile(False)
for name in ("score_layer_5_var0", "score_layer_5_rest", "walk_5_var0", "walk_5_rest",
             "score_layer_6_var0", "score_layer_6_rest", "walk_6_var0", "walk_6_rest", "write_stored"):
    if name in d:
        print(f"{name:20s} {d[name]['total_ms'] / 10:.4f} ms per call", flush=True)
