"""Scoped best-score tables (table_budget_mb): when the dense tables over all
variables exceed the budget, searches build tables per skeleton component
or triplet cluster and every other lookup scans the lists on the device.
The answers must not change: each test forces a budget below the full
tables and compares with the oracle (and checks that the tables were indeed
rebuilt per scope)."""
import numpy as np
import pytest

import synth
import ulg

pytestmark = pytest.mark.gpu


def _costs(o, X, lam, k, cands):
    offs, sets, scores = o.Dataset(X).score_all(lam, cands, k, threads=8)
    costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
    return offs, sets, costs


def _need_kib(offs, sets, scope):
    """KiB of dense tables over the stored sets inside scope (16 B / entry)."""
    tot = 0
    for v in range(len(offs) - 1):
        if not (scope >> v) & 1:
            tot += 1
            continue
        D = 0
        for s in sets[offs[v]:offs[v + 1]]:
            if int(s) & ~scope == 0:
                D |= int(s)
        tot += 1 << bin(D).count("1")
    return tot * 16 / 1024.0


def _table_builds(ctx):
    p = ctx.profile_get("bs_scatter")
    return 0 if p is None else p["count"]


@pytest.fixture
def ctx(ulg_ctx):
    yield ulg_ctx
    ulg_ctx.set_option("table_budget_kb", 0)


def test_list_scan_queries_and_pdb(ctx, oracle_built):
    o = oracle_built
    n = 15
    X, _ = synth.gaussian_sem(n, 2000, 9600)
    offs, sets, costs = _costs(o, X, 1.0, 3, [(1 << n) - 1] * n)   # full tables: 15 x 2^14 x 16 B = 3.75 MiB
    ctx.set_option("table_budget_kb", 1024)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.search_load(offs, sets, costs)
    assert _table_builds(ctx) == 0
    srch = o.Search(n, offs, sets, costs)
    rng = np.random.default_rng(2)
    vs = [int(v) for v in rng.integers(0, n, 3000)]
    Ss = [int(x) for x in rng.integers(0, 1 << n, 3000, dtype=np.int64)]
    gc, gp = ctx.bestscore(vs, Ss)
    for v, S, c, p in zip(vs, Ss, gc, gp):
        ec, ep = srch.bestscore(v, S)
        assert np.float32(c) == np.float32(ec) and int(p) == ep, (v, S)
    # a PDB over all variables: every lookup scans the lists
    srch.pdb_build(2)
    ctx.pdb_build(2)
    Ss = Ss[:2000] + [0, (1 << n) - 1]
    h, comp = ctx.pdb_h(Ss)
    for S, hv, cv in zip(Ss, h, comp):
        eh, ec = srch.pdb_h(S)
        assert np.float32(hv).tobytes() == np.float32(eh).tobytes() and int(cv) == ec
    ctx.profile(False)


def test_exact_astar_per_component_tables(ctx, oracle_built):
    o = oracle_built
    n = 36
    parts = [synth.gaussian_sem(12, 2500, 9601 + b) for b in range(3)]
    X = np.hstack([p[0] for p in parts])
    rows = []
    for b, (_, W) in enumerate(parts):
        for r in synth.true_skeleton_edges(W, 0.3, 9603 + b):
            rows.append(r << (12 * b))
    cands = ulg.candidates_from_edges(rows, n)
    offs, sets, costs = _costs(o, X, 2.0, 4, cands)
    comp = [((1 << 12) - 1) << (12 * b) for b in range(3)]
    budget = max(_need_kib(offs, sets, c) for c in comp) + 1
    assert _need_kib(offs, sets, (1 << n) - 1) > budget
    ctx.set_option("table_budget_kb", int(budget))
    ctx.profile(True)
    ctx.profile_reset()
    ctx.search_load(offs, sets, costs)
    res = ctx.astar(edges=rows, mode=0)
    builds = _table_builds(ctx)
    ctx.profile(False)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows)
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert res["net_text"] == ref["net_text"] and res["expanded"] == ref["expanded"]
    assert builds >= 2, "tables were expected per component"
    with pytest.raises(ulg.ULGError, match="budget"):
        ctx.astar(edges=rows, mode=1)   # the GPU search needs tables over every variable


def test_triplet_per_cluster_tables(ctx, oracle_built):
    o = oracle_built
    n = 22
    X, W = synth.gaussian_sem(n, 3000, 9604)
    rows = synth.true_skeleton_edges(W, 0.12, 9604)
    rows = [r & ~(1 << i) for i, r in enumerate(rows)]
    cands = ulg.candidates_from_edges(rows, n)
    offs, sets, costs = _costs(o, X, 2.0, 3, cands)
    # a budget that holds the tables of every initial triple cluster but not all variables
    cl = [r | (1 << v) for v, r in enumerate(rows)]
    big = max(_need_kib(offs, sets, cl[i] | cl[j] | cl[k])
              for i in range(n) for j in range(i) for k in range(j) if bin(cl[i] | cl[j] | cl[k]).count("1") <= 26)
    budget = 2 * big + 1
    assert _need_kib(offs, sets, (1 << n) - 1) > budget
    ctx.set_option("table_budget_kb", int(budget))
    ctx.profile(True)
    ctx.profile_reset()
    ctx.search_load(offs, sets, costs)
    res = ctx.triplet(edges=rows)
    builds = _table_builds(ctx)
    ctx.profile(False)
    ref = o.triplet(o.Search(n, offs, sets, costs), edges=rows)
    assert res["mec"].tolist() == ref["mec"].tolist()
    assert (res["runs"], res["distinct"], res["expanded"]) == (ref["runs"], ref["distinct"], ref["expanded"])
    assert builds >= 2
