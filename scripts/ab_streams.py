"""Scoring step time vs the number of stream groups (ulg option score_streams)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import numpy as np
import synth, ulg
n, N, k = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (25, 10000, 6)))
groups = [int(x) for x in (sys.argv[4].split(",") if len(sys.argv) > 4 else "1,2,3,4".split(","))]
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
full = [(1 << n) - 1] * n
res = {g: [] for g in groups}
ref = None
for rnd in range(7):
    for g in groups:
        ctx.set_option("score_streams", g)
        t = time.perf_counter(); st, sc = ctx.score(list(range(n)), full, k); dt = time.perf_counter() - t
        res[g].append(dt * 1e3)
        out = ctx.fetch(st)
        h = (out[1].tobytes(), out[2].tobytes())
        if ref is None: ref = h
        assert h == ref, f"score_streams {g} differs"
print(json.dumps({g: float(np.median(v[1:])) for g, v in res.items()}))
