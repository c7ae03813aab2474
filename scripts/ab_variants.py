"""Interleaved A/B timing of the scorer variants at a bench config (one process)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import numpy as np
import synth, ulg
n, N, k = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (25, 10000, 6)))
variants = [int(x) for x in (sys.argv[4].split(",") if len(sys.argv) > 4 else "0,1,2,3".split(","))]
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
full = [(1 << n) - 1] * n
res = {v: [] for v in variants}
ref = None
for rnd in range(5):
    for v in variants:
        ctx.set_option("score_variant", v)
        ctx.profile(True); ctx.profile_reset()
        t = time.perf_counter(); st, sc = ctx.score(list(range(n)), full, k); dt = time.perf_counter() - t
        prof = ctx.profile_dump(); ctx.profile(False)
        res[v].append({"ms": dt * 1e3, f"L{k}rest_ms": prof.get(f"score_layer_{k}_rest", {}).get("total_ms"),
                       "prof": {kk: round(vv.get("total_ms", 0), 4) for kk, vv in prof.items() if vv.get("total_ms", 0) > 0.05}})
        out = ctx.fetch(st)
        h = (out[1].tobytes(), out[2].tobytes())
        if ref is None: ref = h
        assert h == ref, f"variant {v} differs"
print(json.dumps({v: {"median_ms": float(np.median([r["ms"] for r in res[v]])),
                      "median_layer_ms": float(np.median([r[f"L{k}rest_ms"] for r in res[v]])),
                      "last_profile": res[v][-1]["prof"]} for v in variants}, indent=1))
