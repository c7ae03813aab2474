#!/usr/bin/env python3
"""Can the GPU sweep certify the reference's A* DAG without the host replay?

A13 (run_astar_on_one_scc, astar_main.cpp:266-459) returns the DAG of the
first-popped minimiser chain: node T keeps the leaf of the first popped
predecessor that reaches its final g (strict '<' on update, :444), pops go
by (f, deeper first) (node.h:124-135) and exact (f, layer) ties by the
heap's layout (priority_queue-inl.h:19-234).  From the sweep's values
(G = min-plus over all predecessors, F = fl(G + h)) this study builds, for
seeded n=20 cases, the backward closure R of the goal under "minimisers of
the smallest F" (the tie set TS(T)) and checks sufficient conditions under
which EVERY valid heap order (any minimal element popped) gives the same
goal g and DAG:
  (b) minimisers outside TS(T) have F above the running maximum Mpre(T) of
      F along every closure path to TS(T) (they cannot pop first);
  (a) the best non-minimising value gives T an f above Mpre(T) (T cannot be
      popped before a member of TS(T) with a wrong g);
  (dag) every variable gets one parent set over all closure edges;
  plus costs <= 0 and h <= -2 off the goal, so the comparator's FLT_EPSILON
  rule is exact equality and the heap is a valid heap.
The CPU oracle's A* (the reference's heap replayed) is the ground truth.
Test infrastructure only (oracle); results: profiles/r3/cert_study_n20.json.

    python scripts/cert_study.py [first_seed] [count] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import oracle  # noqa: E402
import synth  # noqa: E402

EPS = np.float32(np.finfo(np.float32).eps)


def lists_for(seed, n=20, N=10000, k=4, lam=2.0, threads=8):
    X, _ = synth.gaussian_sem(n, N, seed)
    ds = oracle.Dataset(X)
    offs, sets, scores = ds.score_all(lam, [(1 << n) - 1] * n, k, threads=threads)
    costs = np.array([oracle.quantize(float(x)) for x in scores], dtype=np.float32)
    return offs, sets, costs


def study(offs, sets, costs):
    n = len(offs) - 1
    ALL = (1 << n) - 1
    H = 1 << (n - 1)
    a = np.arange(H)
    bs = []
    for v in range(n):  # getScore(v, .) as a dense subset-min table
        t = np.full(H, np.inf, dtype=np.float32)
        s = sets[offs[v]:offs[v + 1]].astype(np.int64)
        idx = ((s >> (v + 1)) << v) | (s & ((1 << v) - 1))
        np.minimum.at(t, idx, costs[offs[v]:offs[v + 1]])
        for b in range(n - 1):
            hi = a[(a & (1 << b)) != 0]
            t[hi] = np.minimum(t[hi], t[hi ^ (1 << b)])
        bs.append(t)
    srch = oracle.Search(n, offs, sets, costs)
    srch.pdb_build(2)
    groups = srch.pdb_groups()
    masks = np.arange(1 << n, dtype=np.int64)
    pc = np.zeros(1 << n, dtype=np.int64)
    for b in range(n):
        pc += (masks >> b) & 1

    def pext(x, g):
        r, i = np.zeros_like(x), 0
        for b in range(n):
            if (g >> b) & 1:
                r |= ((x >> b) & 1) << i
                i += 1
        return r
    pd = []
    for gi, g in enumerate(groups):
        k = bin(g).count("1")
        rr = np.arange(1 << k)
        R, i = np.zeros(1 << k, dtype=np.int64), 0
        for b in range(n):
            if (g >> b) & 1:
                R |= ((rr >> i) & 1) << b
                i += 1
        pd.append(np.array([oracle.lib().ora_pdb_value(srch.h, gi, int(x)) for x in R], dtype=np.float32))
    rem = (~masks) & ALL
    vs0, vs1 = groups[0] & rem, groups[1] & rem
    p0, p1 = pd[0][pext(vs0, groups[0])], pd[1][pext(vs1, groups[1])]
    # StaticPatternDatabase::h (static_pattern_database.cpp:145-174), two groups
    h = np.where(vs0 == rem, p0, np.where(vs1 == rem, p1, (np.float32(0) + p0).astype(np.float32) + p1))
    h = h.astype(np.float32)
    G = np.full(1 << n, np.inf, dtype=np.float32)
    G[0] = 0
    for L in range(1, n + 1):
        T = masks[pc == L]
        best = np.full(len(T), np.inf, dtype=np.float32)
        for v in range(n):
            sel = ((T >> v) & 1) == 1
            P = T[sel] ^ (1 << v)
            val = (G[P] + bs[v][((P >> (v + 1)) << v) | (P & ((1 << v) - 1))]).astype(np.float32)
            best[sel] = np.minimum(best[sel], val)
        G[T] = best
    F = (G + h).astype(np.float32)

    def val(P, v):
        return np.float32(G[P] + bs[v][((P >> (v + 1)) << v) | (P & ((1 << v) - 1))])
    R, stack, info, par, why = {ALL}, [ALL], {}, {}, {}
    ties = 0
    while stack:
        T = stack.pop()
        if T == 0:
            continue
        vals = [(v, val(T ^ (1 << v), v)) for v in range(n) if (T >> v) & 1]
        mins = [v for v, x in vals if x == G[T]]
        phi = min(F[T ^ (1 << v)] for v in mins)
        TS = [v for v in mins if F[T ^ (1 << v)] == phi]
        ties += len(TS) > 1
        others = [F[T ^ (1 << v)] for v in mins if F[T ^ (1 << v)] != phi]
        nonmin = [x for v, x in vals if x != G[T]]
        F2 = np.float32(min(nonmin) + h[T]) if nonmin else np.float32(np.inf)
        info[T] = (TS, others, F2)
        for v in TS:
            Q = T ^ (1 << v)
            p = srch.bestscore(v, Q)[1]
            if par.setdefault(v, p) != p:
                why["dag"] = why.get("dag", 0) + 1
            if Q not in R:
                R.add(Q)
                stack.append(Q)
    Mx = {0: F[0]}
    for T in sorted(R, key=lambda x: bin(x).count("1")):
        if T == 0:
            continue
        TS, others, F2 = info[T]
        Mpre = max(Mx[T ^ (1 << v)] for v in TS)
        Mx[T] = max(Mpre, F[T])
        if others and not (np.float32(min(others) - Mpre) >= EPS):
            why["b"] = why.get("b", 0) + 1
        if not (np.float32(F2 - Mpre) >= EPS):
            why["a"] = why.get("a", 0) + 1
    if not all(srch.bestscore(v, 0)[0] <= 0 for v in range(n)):
        why["cost>0"] = 1
    if not h[masks != ALL].max() <= -2:
        why["h"] = 1
    ref = srch.astar(edges=[ALL] * n)
    ref_par = [int(x) for x in ref["vpar"]]
    cert = not why
    dag = [par.get(v, 0) for v in range(n)]
    return {"closure_nodes": len(R), "closure_nodes_with_tied_minimisers": ties, "certified": cert,
            "failed_conditions": why, "closure_dag_equals_reference": dag == ref_par,
            "reference_cost_equals_sweep": np.float32(ref["cost"]).tobytes() == np.float32(G[ALL]).tobytes(),
            "reference_expanded": ref["expanded"]}


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 9200
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "r3", "cert_study_n20.json")
    rows = []
    for seed in range(first, first + count):
        t = time.time()
        r = dict(seed=seed, **study(*lists_for(seed)))
        rows.append(r)
        print(json.dumps(r), f"{time.time() - t:.1f}s", flush=True)
    summary = {
        "config": "n=20, N=10000, k=4, lambda=2, full skeleton, synth.gaussian_sem seeds %d..%d" % (first, first + count - 1),
        "certified": sum(r["certified"] for r in rows),
        "certified_and_wrong": sum(r["certified"] and not r["closure_dag_equals_reference"] for r in rows),
        "dag_conflict_in_closure": sum("dag" in r["failed_conditions"] for r in rows),
        "reference_cost_differs_from_sweep_min": sum(not r["reference_cost_equals_sweep"] for r in rows),
        "cases": len(rows), "rows": rows}
    json.dump(summary, open(out, "w"), indent=1)
    print({k: v for k, v in summary.items() if k != "rows"})


if __name__ == "__main__":
    main()
