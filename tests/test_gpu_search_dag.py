"""The DAG the GPU layer search (ULG_ASTAR_GPU, search_gpu.hip) returns.

That mode proves only the optimal order cost against the reference; its DAG
is one optimal DAG, which can differ from the exact-order replay's when
float-tied orders exist.  Since `astar --mode gpu` writes a
netFile from it, these tests pin what it must satisfy on its own:
  * `order` is a permutation of the component and every parent set lies
    before its child in it (so the DAG is acyclic);
  * each parent set is what SparseParentList::getScore/getParents returns
    for the prefix (ulg_bestscore_query, sparse_parent_list.cpp:44-55), and
    the float sum of those costs in path order is the goal cost bit for bit
    (the sweep's g(T) = fl(g(T \\ leaf) + bs(leaf, T \\ leaf)),
    astar_main.cpp:327);
  * the goal cost equals the exact-order A*'s within 1e-6 relative.
How often its DAG equals the exact-order DAG is measured and written to
gpurun_out/dag_agreement_<case>.json (not asserted)."""
import json
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _report(name, data):
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"dag_agreement_{name}.json"), "w") as f:
        json.dump(data, f, indent=1)


def check_gpu_dag(ctx, comp, res, n, skip_var0=False):
    """Validate a GPU-mode result on component `comp` (the last one searched)."""
    m = bin(comp).count("1")
    order = [int(x) for x in res["order"][:m]]
    assert sorted(order) == [v for v in range(n) if (comp >> v) & 1]
    prefix, vs, Ss = 0, [], []
    for v in order:
        prefix |= 1 << v
        vs.append(v)
        Ss.append(prefix)
    costs, parents = ctx.bestscore(vs, Ss)
    g = np.float32(0.0)
    before = 0
    for i, v in enumerate(order):
        p = int(parents[i])
        assert p & ~before == 0, (v, p, before)  # parents precede the child: acyclic
        if not (skip_var0 and v == 0):
            assert int(res["vpar"][v]) == p, (v, int(res["vpar"][v]), p)
        g = np.float32(g + np.float32(costs[i]))
        before |= 1 << v
    assert g.tobytes() == np.float32(res["cost"]).tobytes(), (float(g), res["cost"])


def _pipeline(ctx, X, k, edges=None):
    import ulg
    n = X.shape[1]
    ctx.load(X, 2.0)
    cands = ulg.candidates_from_edges(edges, n) if edges is not None else [(1 << n) - 1] * n
    ctx.score(list(range(n)), cands, k)
    ctx.search_from_scores()
    full = edges if edges is not None else [(1 << n) - 1] * n
    ex = ctx.astar(edges=full, mode=0, net_text=False)
    gp = ctx.astar(edges=full, mode=1, net_text=False)
    return ex, gp


def test_gpu_dag_valid_c2_and_agreement_over_30_seeds(ulg_ctx):
    """C2 (seed 9200) and 29 more seeded n=20, N=10k, k=4 datasets."""
    n, N, k = 20, 10000, 4
    rows = []
    for seed in range(9200, 9230):
        X, _ = synth.gaussian_sem(n, N, seed)
        ex, gp = _pipeline(ulg_ctx, X, k)
        check_gpu_dag(ulg_ctx, (1 << n) - 1, gp, n)
        assert abs(gp["cost"] - ex["cost"]) <= 1e-6 * abs(ex["cost"])
        rows.append({"seed": seed, "same_dag": [int(x) for x in gp["vpar"]] == [int(x) for x in ex["vpar"]],
                     "same_order": list(gp["order"]) == list(ex["order"]),
                     "same_cost_bits": np.float32(gp["cost"]).tobytes() == np.float32(ex["cost"]).tobytes()})
    _report("n20", {"config": "n=20, N=10000, k=4, lambda=2, full skeleton, seeds 9200..9229",
                    "same_dag": sum(r["same_dag"] for r in rows),
                    "same_cost_bits": sum(r["same_cost_bits"] for r in rows),
                    "cases": len(rows), "rows": rows})


def test_gpu_dag_valid_sparse_components(ulg_ctx):
    """Two skeleton components with the neighbour filter (the last component
    is what the outputs hold, astar_main.cpp:470,519; vpar[0] is the
    reference's reconstruct quirk there, so it is not compared)."""
    n = 14
    X1, W1 = synth.gaussian_sem(8, 2500, 9320)
    X2, W2 = synth.gaussian_sem(6, 2500, 9321)
    X = np.hstack([X1, X2])
    W = np.zeros((n, n))
    W[:8, :8] = W1
    W[8:, 8:] = W2
    rows = synth.true_skeleton_edges(W)
    ex, gp = _pipeline(ulg_ctx, X, 3, rows)
    check_gpu_dag(ulg_ctx, ((1 << n) - 1) & ~0xff, gp, n, skip_var0=True)
    assert abs(gp["cost"] - ex["cost"]) <= 1e-6 * abs(ex["cost"])


def test_gpu_dag_valid_connected_sparse_skeleton(ulg_ctx):
    n = 18
    X, W = synth.gaussian_sem(n, 5000, 9340)
    rows = synth.true_skeleton_edges(W, extra_frac=0.3, seed=2)
    # one component: join any stragglers to variable 0
    reach, fr = 1, 1
    while fr:
        nb = 0
        for v in range(n):
            if (fr >> v) & 1:
                nb |= rows[v]
        fr = nb & ~reach
        reach |= nb
    for v in range(n):
        if not (reach >> v) & 1:
            rows[v] |= 1
            rows[0] |= 1 << v
    ex, gp = _pipeline(ulg_ctx, X, 5, rows)
    check_gpu_dag(ulg_ctx, (1 << n) - 1, gp, n)
    assert abs(gp["cost"] - ex["cost"]) <= 1e-6 * abs(ex["cost"])


def _block_skeleton(n, blocks):
    """Complete skeleton rows on each block of variables (no filter inside a
    component, so the sweep-table launches run per component)."""
    rows = [0] * n
    for b in blocks:
        m = sum(1 << v for v in b)
        for v in b:
            rows[v] = m
    return rows


@pytest.mark.parametrize("case", ["full", "blocks", "scoped"])
def test_sweep_table_gives_identical_search(ulg_ctx, case):
    """ulg_set_option("sweep_table"): the (variable, layer, colex) cost slices
    hold exactly getScore's floats, so the sweep with and without them returns
    the same goal cost bits, order and parent sets -- on a full skeleton, on
    complete blocks (components whose variables are not 0..m-1, so the slices
    map compact positions back through the component), and on those blocks
    with a table budget below the all-variable tables (tables built per
    component, scope != every variable)."""
    import ulg
    n, N, k = 20, 8000, 4
    X, _ = synth.gaussian_sem(n, N, 9360)
    if case in ("blocks", "scoped"):
        edges = _block_skeleton(n, [[0, 3, 5, 6, 9, 12, 13, 17, 19], [1, 2, 4, 7, 8, 10, 11, 14, 15, 16, 18]])
    else:
        edges = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), ulg.candidates_from_edges(edges, n), k)
    if case == "scoped":
        ulg_ctx.set_option("table_budget_kb", 4096)  # all-variable tables: 120 MiB
    try:
        ulg_ctx.search_from_scores()
        res = []
        for on in (0, 1, 1, 2):  # the second 1 reuses the cached slices; 2 = 64-bit index arithmetic
            ulg_ctx.set_option("sweep_table", on)
            res.append(ulg_ctx.astar(edges=edges, mode=1, net_text=False))
    finally:
        ulg_ctx.set_option("sweep_table", 1)
        ulg_ctx.set_option("table_budget_kb", 0)
    for r in res[1:]:
        assert np.float32(r["cost"]).tobytes() == np.float32(res[0]["cost"]).tobytes()
        assert [int(x) for x in r["order"]] == [int(x) for x in res[0]["order"]]
        assert [int(x) for x in r["vpar"]] == [int(x) for x in res[0]["vpar"]]
        assert r["expanded"] == res[0]["expanded"]
    ex = ulg_ctx.astar(edges=edges, mode=0, net_text=False)
    assert abs(res[1]["cost"] - ex["cost"]) <= 1e-6 * abs(ex["cost"])
