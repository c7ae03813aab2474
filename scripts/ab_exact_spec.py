#!/usr/bin/env python3
"""A/B of the exact-order replay's prefetch modes at C3 (or C2) in one
process: the tables and successor-cost rows are built once, then the replay
runs alternately under each ULG_EXACT_PF value (read per call).  Every run's
expansions and goal cost must agree.

    python scripts/ab_exact_spec.py [--config c3] [--modes 6 22] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

CFG = {"c2": (20, 10000, 4), "c3": (25, 10000, 6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--modes", nargs="+", default=["6", "22"])
    ap.add_argument("--deep", nargs="+", default=["6"], help="ULG_EXACT_SPEC_DEEP values (spec modes only)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--settled", nargs="+", default=None, help="exact_settled values to alternate (pf modes: first only)")
    a = ap.parse_args()
    n, N, k = CFG[a.config]
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), full, k)
    ctx.search_from_scores()
    t = time.perf_counter()
    r0 = ctx.astar(edges=full, mode=0, net_text=False)
    print(json.dumps({"first_call_s": time.perf_counter() - t, "expanded": r0["expanded"], "cost": r0["cost"]}),
          flush=True)
    if a.settled:
        res = {f"settled={v}": [] for v in a.settled}
        keys = list(res)
        for rep in range(a.reps):
            for v in a.settled:
                v, _, pf = v.partition("/")  # "1/134": exact_settled 1 under ULG_EXACT_PF 134
                os.environ["ULG_EXACT_PF"] = pf or "6"
                ctx.set_option("exact_settled", int(v))
                ctx.astar(edges=full, mode=0, net_text=False)  # rebuilds the rows for this setting
                t = time.perf_counter()
                r = ctx.astar(edges=full, mode=0, net_text=False)
                dt = time.perf_counter() - t
                assert r["expanded"] == r0["expanded"] and r["cost"] == r0["cost"], (v, r["expanded"], r["cost"])
                assert [int(x) for x in r["vpar"]] == [int(x) for x in r0["vpar"]] and list(r["order"]) == list(r0["order"])
                res[keys[a.settled.index(v + ("/" + pf if pf else ""))]].append(round(dt, 3))
                print(json.dumps({"rep": rep, "exact_settled": v, "s": round(dt, 3),
                                  "expansions_per_s": r["expanded"] / dt}), flush=True)
        print(json.dumps({"config": a.config, "seconds": res}), flush=True)
        ctx.close()
        return
    arms = []
    for m in a.modes:
        if int(m) & 16:
            arms += [(m, f) for f in a.deep]
        else:
            arms.append((m, None))
    res = {f"{m}/{f}": [] for m, f in arms}
    for rep in range(a.reps):
        for m, f in arms:
            os.environ["ULG_EXACT_PF"] = m
            if f is not None:
                os.environ["ULG_EXACT_SPEC_DEEP"] = f
            t = time.perf_counter()
            r = ctx.astar(edges=full, mode=0, net_text=False)
            dt = time.perf_counter() - t
            assert r["expanded"] == r0["expanded"] and r["cost"] == r0["cost"], (m, f, r["expanded"], r["cost"])
            res[f"{m}/{f}"].append(round(dt, 3))
            print(json.dumps({"rep": rep, "pf": m, "deep": f, "s": round(dt, 3),
                              "expansions_per_s": r["expanded"] / dt}), flush=True)
    print(json.dumps({"config": a.config, "seconds": res}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
