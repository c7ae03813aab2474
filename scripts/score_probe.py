#!/usr/bin/env python3
"""Single synchronised scoring calls on a few configurations: the time of one
call (median / min of --reps), a digest of the stored lists (sets and score
bits) so builds and options can be compared run against run, a determinism
check (a second call, graph replay included, gives the same lists) and, at
C3, the oracle command lines' per-variable digests (tests/golden/c3_oracle.json).

    python scripts/score_probe.py [--cases small c2 c3 c5] [--reps 10] [--options name=value,...] [--lib path]
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
import synth  # noqa: E402
import ulg  # noqa: E402

CASES = {
    "small": [(11, 2500, 6, "full"), (12, 3000, 6, "novar0"), (9, 2000, 4, "full"), (14, 3000, 5, "sparse")],
    "c2": [(20, 10000, 4, "full")],
    "c3": [(25, 10000, 6, "full")],
    "c5": [(32, 50000, 6, "full")],
}


def cands_for(n, kind, seed):
    full = (1 << n) - 1
    if kind == "full":
        return list(range(n)), [full] * n
    if kind == "novar0":
        return list(range(1, n)), [full & ~1] * (n - 1)
    rng = np.random.default_rng(seed)
    c = [int(full & ~int(rng.integers(0, 1 << n))) | 1 for _ in range(n)]
    return list(range(n)), c


def digest(res):
    h = hashlib.sha256()
    for x in res:
        h.update(np.asarray(x).tobytes())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["small", "c2", "c3", "c5"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--options", default="")
    ap.add_argument("--lib", default=None, help="another build of libulg.so (timing experiments)")
    a = ap.parse_args()
    if a.lib:
        ulg.LIB_PATH = os.path.abspath(a.lib)
    ctx = ulg.Context(0)
    for kv in filter(None, a.options.split(",")):
        k_, v_ = kv.split("=")
        ctx.set_option(k_, int(v_))
    ok = True
    for name in a.cases:
        for (n, N, k, kind) in CASES[name]:
            X, _ = synth.gaussian_sem(n, N, 9200)
            ctx.load(X, 2.0)
            variables, cands = cands_for(n, kind, n)
            st, _ = ctx.score(variables, cands, k)
            res = ctx.fetch(st)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                ctx.score(variables, cands, k)
                ts.append(time.perf_counter() - t0)
            st2, _ = ctx.score(variables, cands, k)
            same = digest(ctx.fetch(st2)) == digest(res)
            ok &= same
            oracle_ok = None
            if name == "c3":
                ref = json.load(open(os.path.join(ROOT, "tests", "golden", "c3_oracle.json")))
                offs, sets = res[0], res[1]
                oracle_ok = all(
                    hashlib.sha256(np.sort(np.asarray(sets[offs[v]:offs[v + 1]]).astype(np.uint64)).tobytes())
                    .hexdigest() == ref["sets_sha256_per_variable"][v] for v in range(n))
                ok &= oracle_ok
            print(json.dumps({"case": name, "n": n, "N": N, "k": k, "kind": kind, "stored": int(res[0][-1]),
                              "digest": digest(res), "deterministic": same, "c3_oracle": oracle_ok,
                              "ms_median": 1e3 * float(np.median(ts)), "ms_min": 1e3 * float(np.min(ts)),
                              "options": a.options, "lib": a.lib}), flush=True)
    ctx.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
