#!/usr/bin/env python3
"""Scoring steps in flight: one context scoring synchronously step after
step against S contexts (same data) whose calls are queued with
ulg_cbic_score_async and collected S - 1 steps later.  Every step scores
the whole share; the lists of every slot must equal the synchronous ones.
Prints ms per step for the whole C3 call and for each rank share of
shard.assign over --ranks.

    python scripts/slots_probe.py [--slots 2 3] [--ranks 8] [--steps 40]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import numpy as np  # noqa: E402
import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402


def digest(ctx, stored):
    offs, sets, scores = ctx.fetch(stored)
    h = hashlib.sha256()
    for a in (offs, sets, scores):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def run(ctxs, part, cands, k, steps):
    S = len(ctxs)
    pend = []
    t = time.perf_counter()
    for i in range(steps):
        c = ctxs[i % S]
        if S == 1:
            c.score(part, cands, k)
            continue
        c.score_async(part, cands, k)
        pend.append(c)
        if len(pend) == S:
            pend.pop(0).score_finish()
    for c in pend:
        c.score_finish()
    return (time.perf_counter() - t) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--options", default="", help="ulg_set_option name=value,... on every context")
    a = ap.parse_args()
    n, N, k = 25, 10000, 6
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ctxs = []
    for _ in range(max(a.slots)):
        c = ulg.Context(0)
        for kv in filter(None, a.options.split(",")):
            x, y = kv.split("=")
            c.set_option(x, int(y))
        c.load(X, 2.0)
        ctxs.append(c)
    shares = [("whole", list(range(n)))]
    parts = shard.assign(n, a.ranks, full, k)
    shares += [(f"rank{r}of{a.ranks}", list(p)) for r, p in enumerate(parts)]
    out = {}
    for name, part in shares:
        cands = [full[v] for v in part]
        res = {}
        ref = None
        for S in [1] + a.slots:
            run(ctxs[:S], part, cands, k, 6)  # warm-up (graph capture per context)
            res[S] = min(run(ctxs[:S], part, cands, k, a.steps) for _ in range(3))
            for c in ctxs[:S]:
                st, _ = c.score_finish()
                d = digest(c, st)
                assert ref is None or d == ref, (name, S, "lists differ")
                ref = d
        out[name] = {f"slots{S}_ms_per_step": round(v, 4) for S, v in res.items()}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
