#!/usr/bin/env python3
"""The persistent scoring pipeline (score_pipe 1, cbic_pipe.hip) against the
layer launches (score_pipe 0): identical lists on every case, and the time of
one synchronised call each (median of --reps).

    python scripts/pipe_probe.py [--cases c2 c3 c5 small] [--reps 10] [--options name=value,...]
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


def timed(ctx, variables, cands, k, reps):
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        ctx.score(variables, cands, k)
        ts.append(time.perf_counter() - a)
    return 1e3 * float(np.median(ts)), 1e3 * float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["small", "c2", "c3", "c5"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--options", default="")
    ap.add_argument("--lib", default=None, help="another build of libulg.so (timing experiments)")
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 1], help="score_pipe values to run (0: layers only)")
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
            res, ms = {}, {}
            for pipe in a.modes:  # the context default is whatever ulg_internal.h says
                ctx.set_option("score_pipe", pipe)
                st, _ = ctx.score(variables, cands, k)
                res[pipe] = ctx.fetch(st)
                ms[pipe] = timed(ctx, variables, cands, k, a.reps)
                st2, _ = ctx.score(variables, cands, k)
                again = ctx.fetch(st2)
                if any(np.asarray(x).tobytes() != np.asarray(y).tobytes() for x, y in zip(res[pipe], again)):
                    print(json.dumps({"case": name, "n": n, "pipe": pipe, "error": "not deterministic"}), flush=True)
                    ok = False
            m0, m1 = a.modes[0], a.modes[-1]
            same = all(np.asarray(x).tobytes() == np.asarray(y).tobytes() for x, y in zip(res[m0], res[m1]))
            ok &= same
            if name == "c3":  # against the oracle command lines' digests too
                import hashlib
                ref = json.load(open(os.path.join(ROOT, "tests", "golden", "c3_oracle.json")))
                offs, sets = res[m1][0], res[m1][1]
                for v in range(n):
                    srt = np.sort(np.asarray(sets[offs[v]:offs[v + 1]]).astype(np.uint64))
                    if hashlib.sha256(srt.tobytes()).hexdigest() != ref["sets_sha256_per_variable"][v]:
                        print(json.dumps({"case": name, "error": f"variable {v} differs from c3_oracle.json"}))
                        ok = False
            print(json.dumps({"case": name, "n": n, "N": N, "k": k, "kind": kind, "identical": same,
                              "stored": int(res[m1][0][-1]), "layers_ms": ms.get(0), "pipe_ms": ms.get(1),
                              "options": a.options, "sliced_k": os.environ.get("ULG_SLICED_K")}), flush=True)
    ctx.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
