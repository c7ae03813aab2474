#!/usr/bin/env python3
"""C4 (n=30, N=100k, MMPC skeleton, 2-hop candidates, -p 29) on one GPU:
where the scoring step's time goes, and how well shard.assign balances it.

  1. every variable scored alone (best of 3, warm): its time, m_v, sets;
  2. the whole step (all 30 variables in one call, as bench.py --config c4
     runs it): best of 3, and one profiled call's per-kernel totals;
  3. for 2, 4 and 8 ranks, each rank's share from shard.assign scored alone
     (best of 3): max over ranks / the whole step -- the strong-scaling bound
     the partition allows (the ranks run on separate GPUs at N > 1).

    python scripts/c4_balance.py [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402


def best_of(fn, reps=3):
    fn()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    n, N, k = 30, 100000, 29
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx = ulg.Context(0)
    for kv in filter(None, os.environ.get("ULG_OPTS", "").split(",")):  # A/B knobs: name=value,...
        a, b = kv.split("=")
        ctx.set_option(a, int(b))
    ctx.load(X, 2.0)
    cands = ulg.candidates_from_edges(ctx.mmpc(0.01), n)
    m = [bin(c & ~(1 << v)).count("1") for v, c in enumerate(cands)]
    per_var = {}
    for v in range(n):
        per_var[v] = best_of(lambda: ctx.score([v], [cands[v]], k))
        print(f"v={v:2d} m={m[v]:2d} sets={shard.var_weight(n, v, cands[v], k):8d} {per_var[v] * 1e3:8.2f} ms",
              flush=True)
    allv = list(range(n))
    full = best_of(lambda: ctx.score(allv, cands, k))
    ctx.profile(True)
    ctx.profile_select(None)
    ctx.profile_reset()
    ctx.score(allv, cands, k)
    kern = ctx.profile_dump()
    ctx.profile(False)
    top = sorted(((a, b["total_ms"]) for a, b in kern.items()), key=lambda x: -x[1])[:12]
    print(f"whole step {full * 1e3:.2f} ms; kernels: " + " ".join(f"{a}={b:.2f}" for a, b in top), flush=True)
    out = {"config": "C4: n=30, N=100000, MMPC alpha 0.01, 2-hop candidates, -p 29, lambda 2, seed 9200",
           "whole_step_ms": 1e3 * full, "sum_of_variables_alone_ms": 1e3 * sum(per_var.values()),
           "per_variable_ms": {v: round(1e3 * t, 3) for v, t in per_var.items()}, "m": m,
           "kernel_ms_one_step": {a: round(b, 3) for a, b in top}, "ranks": {}}
    for ws in (2, 4, 8):
        parts = shard.assign(n, ws, cands, k)
        times = [best_of(lambda p=p: ctx.score(p, [cands[v] for v in p], k)) for p in parts]
        out["ranks"][ws] = {"parts": parts, "rank_ms": [round(1e3 * t, 3) for t in times],
                            "max_rank_over_whole": max(times) / full}
        print(f"ws={ws}: rank ms {[round(1e3 * t, 2) for t in times]}, max/whole {max(times) / full:.3f}",
              flush=True)
    ctx.close()
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
