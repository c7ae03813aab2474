#!/usr/bin/env python3
"""A/B of wide-layer options on the whole C4 scoring step (n=30, N=100k, MMPC
alpha 0.01, 2-hop candidates, -p 29, all 30 variables in one call, as
bench.py --config c4): best of 5 per combination, alternating, with a digest
of the lists (which must not depend on the options).

    python scripts/c4_opts_ab.py "wide_host=4096,wide_host_threads=8" "wide_host=1024" ...
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

args = sys.argv[1:]
ctx = ulg.Context(0)
reps = 5
if args and args[0] == "--c1":  # C1 at the reference's defaults instead: hepatitis, lambda 0.5, -p 19
    args = args[1:]
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_wide import load_csv_ascii
    X = load_csv_ascii(os.path.join(ROOT, "tests", "golden", "hepatitis.clean.csv"))
    n = X.shape[1]
    k = n - 1
    ctx.load(X, 0.5)
    cands = [(1 << n) - 1] * n
    reps = 1
else:
    n, N, k = 30, 100000, 29
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx.load(X, 2.0)
    cands = ulg.candidates_from_edges(ctx.mmpc(0.01), n)
combos = args or ["wide_host=4096"]
for rnd in range(2):
    for combo in combos:
        for kv in filter(None, combo.split(",")):
            a, b = kv.split("=")
            ctx.set_option(a, int(b))
        stored, _ = ctx.score(list(range(n)), cands, k)
        h = hashlib.sha256()
        for arr in ctx.fetch(stored):
            h.update(np.ascontiguousarray(arr).tobytes())
        best = 1e9
        for _ in range(reps):
            t = time.perf_counter()
            ctx.score(list(range(n)), cands, k)
            best = min(best, time.perf_counter() - t)
        print(f"{combo}: {best * 1e3:.2f} ms, {stored} stored, digest {h.hexdigest()[:16]}", flush=True)
ctx.close()
