"""A/B of one scorer option (ulg_set_option NAME=value, alternating values
in one process): best-of-3 wall time per scoring call (100 calls, graph
replay, no profiling) and a digest of the stored lists, which must not
depend on the option.  C3 by default; `--all` adds C2 and C5.
  OPTION=score_small_split VALUES=0,1 python scripts/score_opt_ab.py --all"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

OPT = os.environ.get("OPTION", "score_small_split")
VALUES = [int(x) for x in os.environ.get("VALUES", "0,1").split(",")]


def digest(ctx, stored):
    h = hashlib.sha256()
    for a in ctx.fetch(stored):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def run(name, X, variables, cands, k, reps=100, rounds=2):
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    for _ in range(rounds):
        for val in VALUES:
            ctx.set_option(OPT, val)
            for _ in range(3):
                stored, scored = ctx.score(variables, cands, k)
            dg = digest(ctx, stored)
            best = 1e9
            for _ in range(3):
                t = time.perf_counter()
                for _ in range(reps):
                    ctx.score(variables, cands, k)
                best = min(best, (time.perf_counter() - t) / reps)
            print(f"{name} {OPT}={val}: {best * 1e3:.4f} ms per call, {stored} of {scored} stored, digest {dg}",
                  flush=True)
            if os.environ.get("PROFILE") == "1":
                # per-kernel times of one profiled call (HIP events, eager launches)
                ctx.profile(True)
                ctx.profile_select(None)
                ctx.profile_reset()
                ctx.score(variables, cands, k)
                kern = ctx.profile_dump()
                ctx.profile(False)
                print("   ", " ".join(f"{kk}={v['total_ms']:.4f}" for kk, v in sorted(kern.items())
                                      if v["total_ms"] >= 0.01), flush=True)
    ctx.close()


X, _ = synth.gaussian_sem(25, 10000, 9200)
run("c3", X, list(range(25)), [(1 << 25) - 1] * 25, 6)
if "--all" in sys.argv:
    X, _ = synth.gaussian_sem(20, 10000, 9100)
    run("c2", X, list(range(20)), [(1 << 20) - 1] * 20, 4)
    X, _ = synth.gaussian_sem(32, 50000, 9300)
    run("c5", X, list(range(32)), [(1 << 32) - 1] * 32, 6, reps=10, rounds=1)
