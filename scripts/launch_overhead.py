"""Scoring-call latency at tiny layer counts (C3 data, k = 1..6): where the
per-layer launch/dependency overhead shows against the kernels' work."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth, ulg
n, N = 25, 10000
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
full = [(1 << n) - 1] * n
for streams, small in [tuple(int(x) for x in a.split(",")) for a in (sys.argv[1:] or ["3,4"])]:
    ctx.set_option("score_streams", streams)
    ctx.set_option("score_small_layers", small)
    for k in range(5, 7):
        for _ in range(3):
            ctx.score(list(range(n)), full, k)
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            st, sc = ctx.score(list(range(n)), full, k)
        dt = (time.perf_counter() - t0) / reps
        print(f"streams={streams} small={small} k={k}: {sc} sets, {1e3 * dt:.3f} ms per call", flush=True)
