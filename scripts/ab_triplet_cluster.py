#!/usr/bin/env python3
"""Times single triplet_astar cluster searches (the re-opening exact replay)
of the C5 sparse run (scripts/c5_triplet.py --extra 0.0) alone on one host
thread, alternating ULG_EXACT_PF modes; the memo is dropped before every run
(search_from_scores) and every run's expansions and parents must agree.

    python scripts/ab_triplet_cluster.py [--clusters 0xcfed7ffe ...] [--modes 6 22] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import numpy as np  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    # the two longest waits of profiles/r3/r3r_c5_sparse_triplet_trace.log
    ap.add_argument("--clusters", nargs="+", default=["0xcfed7ffe", "0xc7ddfdfe"])
    ap.add_argument("--modes", nargs="+", default=["6", "22"])
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    n, N, k = 32, 50000, 6
    X, W = synth.gaussian_sem(n, N, 9700)
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    rows = [r & ~(1 << i) for i, r in enumerate(synth.true_skeleton_edges(W, 0.0, 9700))]
    ctx.score(list(range(n)), ulg.candidates_from_edges(rows, n), k)
    os.environ["ULG_TRIPLET_THREADS"] = "2"  # > 1: host cost table; a batch of one runs on the caller
    ref = {}
    out = {}
    for rep in range(a.reps):
        for cl in a.clusters:
            for m in a.modes:
                ctx.search_from_scores()
                os.environ["ULG_EXACT_PF"] = m
                t = time.perf_counter()
                par, st = ctx.triplet_solve([int(cl, 16)])
                dt = time.perf_counter() - t
                key = (cl, st["expanded"], bytes(par.tobytes()))
                if cl in ref:
                    assert ref[cl] == key, (cl, m, "result differs")
                ref[cl] = key
                out.setdefault(f"{cl}/pf{m}", []).append(round(dt, 3))
                print(json.dumps({"rep": rep, "cluster": cl, "variables": bin(int(cl, 16)).count("1"), "pf": m,
                                  "expanded": st["expanded"], "s": round(dt, 3),
                                  "expansions_per_s": st["expanded"] / dt}), flush=True)
    print(json.dumps({"seconds": out}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
