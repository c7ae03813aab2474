#!/usr/bin/env python3
"""Strong-scaling bound of the sharded scoring step on one GPU: for 1, 2, 4
and 8 ranks, each rank's shard.assign share (bench.py --mode shard) is scored
alone (best of 5, warm) and, for the largest share, the exchange block is
filled from the scorer's buffers (ListExchange.fill without the collective).
max over ranks / the whole step is what the partition allows before the
all-gather.

    python scripts/share_probe.py [--config c3] [--options name=value,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402

CFG = {"c2": (20, 10000, 4), "c3": (25, 10000, 6), "c5": (32, 50000, 6)}


def best_of(fn, reps=5):
    fn()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--options", default="")
    a = ap.parse_args()
    n, N, k = CFG[a.config]
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx = ulg.Context(0)
    for kv in filter(None, a.options.split(",")):
        x, y = kv.split("=")
        ctx.set_option(x, int(y))
    ctx.load(X, 2.0)
    cands = [(1 << n) - 1] * n
    out = {"config": a.config, "options": a.options}
    whole = best_of(lambda: ctx.score(list(range(n)), cands, k))
    out["whole_ms"] = whole * 1e3
    for ws in (2, 4, 8):
        parts = shard.assign(n, ws, cands, k)
        t = []
        for p in parts:
            t.append(best_of(lambda: ctx.score(list(p), [cands[v] for v in p], k)) * 1e3)
        out[f"ranks{ws}"] = {"share_ms": [round(x, 4) for x in t], "max_over_whole": max(t) / (whole * 1e3),
                             "ideal": 1.0 / ws}
        print(json.dumps({ws: out[f"ranks{ws}"]}), flush=True)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
