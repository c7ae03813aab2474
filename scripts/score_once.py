"""One C3-sized scoring call (diagnostics driver for the env knobs)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth, ulg
n, N, k = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (25, 10000, 6)))
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
for _ in range(2):
    ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
