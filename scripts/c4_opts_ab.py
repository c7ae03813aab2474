#!/usr/bin/env python3
"""C4 (n=30, N=100k, MMPC skeleton, 2-hop candidates, -p 29) whole-step
time under option sets, alternating, lists compared with the first set's.

    python scripts/c4_opts_ab.py "" "wide_host_q=15" ... [--reps 8]
"""
import argparse
import hashlib
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
    ap.add_argument("sets", nargs="+")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    n, N = 30, 100000
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctxs = []
    for opts in a.sets:
        c = ulg.Context(0)
        for kv in filter(None, opts.split(",")):
            k_, v_ = kv.split("=")
            c.set_option(k_, int(v_))
        c.load(X, 2.0)
        ctxs.append(c)
    rows = ctxs[0].mmpc(0.01)
    cands = ulg.candidates_from_edges(rows, n)
    ref = None
    for rnd in range(a.rounds):
        for opts, c in zip(a.sets, ctxs):
            st, _ = c.score(list(range(n)), cands, 29)
            st, _ = c.score(list(range(n)), cands, 29)
            h = hashlib.sha256(b"".join(np.asarray(x).tobytes() for x in c.fetch(st))).hexdigest()[:16]
            ref = ref or h
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                c.score(list(range(n)), cands, 29)
                ts.append(time.perf_counter() - t0)
            print(f"round {rnd} opts '{opts}': median {1e3 * np.median(ts):.1f} ms min {1e3 * np.min(ts):.1f} ms "
                  f"lists {h} {'same' if h == ref else 'DIFFERENT'}", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
