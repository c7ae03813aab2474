"""GPU parity tests of the search side: best-score lattice tables, the static
pattern database, the exact-order A* (bit-exact DAG, cost and expansion
count against the oracle and the reference's golden DAGs) and the GPU
order-graph search (optimal cost)."""
import numpy as np
import pytest

from conftest import fig_dag, load_fig
import synth

pytestmark = pytest.mark.gpu


def _oracle_pipeline(oracle, X, lam, k, cands=None):
    n = X.shape[1]
    ds = oracle.Dataset(X)
    if cands is None:
        cands = [(1 << n) - 1] * n
    offs, sets, scores = ds.score_all(lam, cands, k, threads=8)
    costs = np.array([oracle.quantize(float(s)) for s in scores], dtype=np.float32)
    return offs, sets, scores, costs


def _random_subsets(rng, n, count):
    return [int(x) for x in rng.integers(0, 1 << n, count, dtype=np.int64)]


def test_bestscore_tables_match_list_scan(ulg_ctx, oracle_built):
    o = oracle_built
    n = 12
    X, _ = synth.gaussian_sem(n, 2000, 9300)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, 4)
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    rng = np.random.default_rng(5)
    vs = [int(v) for v in rng.integers(0, n, 6000)]
    Ss = _random_subsets(rng, n, 6000)
    Ss[:n] = [0] * n
    vs[:n] = list(range(n))
    gc, gp = ulg_ctx.bestscore(vs, Ss)
    for v, S, c, p in zip(vs, Ss, gc, gp):
        ec, ep = srch.bestscore(v, S)
        assert np.float32(c) == np.float32(ec), (v, S, c, ec)
        assert int(p) == ep, (v, S, p, ep)


def test_bestscore_tables_heterogeneous_supports(ulg_ctx, oracle_built):
    """Supports of very different sizes (6..19 candidate parents, as a sparse
    skeleton's 2-hop sets give): per-variable tables start at offsets that are
    not aligned to their own size, and m > 14 exercises the strided zeta pass."""
    o = oracle_built
    n = 20
    X, _ = synth.gaussian_sem(n, 2000, 9302)
    rng = np.random.default_rng(11)
    cands = []
    for v in range(n):
        others = [u for u in range(n) if u != v]
        m = [6, 19, 9, 15, 17, 7, 16, 12, 18, 8, 14, 19, 6, 11, 15, 10, 17, 13, 9, 16][v]
        pick = rng.choice(others, size=m, replace=False)
        cands.append(int(sum(1 << int(u) for u in pick)))
    offs, sets, scores, costs = _oracle_pipeline(o, X, 0.5, 2, cands)
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    vs = [int(v) for v in rng.integers(0, n, 20000)]
    Ss = _random_subsets(rng, n, 20000)
    gc, gp = ulg_ctx.bestscore(vs, Ss)
    for v, S, c, p in zip(vs, Ss, gc, gp):
        ec, ep = srch.bestscore(v, S)
        assert np.float32(c) == np.float32(ec), (v, S, c, ec)
        assert int(p) == ep, (v, S, p, ep)


@pytest.mark.parametrize("n,k", [(16, 2), (25, 2), (20, 4)])
def test_bestscore_big_tables_register_zeta(ulg_ctx, oracle_built, n, k):
    """Tables of >= 2^14 entries per variable take the sorted-entries tile
    build and the register-blocked subset-min (pass A for every m >= 14, pass
    B when a variable has 10 bits above bit 14: n = 25 gives m = 24)."""
    o = oracle_built
    X, _ = synth.gaussian_sem(n, 2000, 9303 + n)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 0.5, k)
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    rng = np.random.default_rng(n)
    vs = [int(v) for v in rng.integers(0, n, 20000)]
    Ss = _random_subsets(rng, n, 20000)
    # subsets near the top and the bottom of the lattice as well
    Ss[:64] = [(1 << n) - 1 - (1 << int(b)) for b in rng.integers(0, n, 64)]
    Ss[64:128] = [1 << int(b) for b in rng.integers(0, n, 64)]
    gc, gp = ulg_ctx.bestscore(vs, Ss)
    for v, S, c, p in zip(vs, Ss, gc, gp):
        ec, ep = srch.bestscore(v, S)
        assert np.float32(c) == np.float32(ec), (v, S, c, ec)
        assert int(p) == ep, (v, S, p, ep)


def test_bestscore_ties_fall_to_file_order(ulg_ctx, oracle_built):
    """Equal costs: the first set in file order wins (pinned N7)."""
    o = oracle_built
    n = 5
    offs = np.array([0, 4, 5, 6, 7, 8], dtype=np.int64)
    sets = np.array([0b00110, 0b01000, 0b00010, 0, 0, 0, 0, 0], dtype=np.uint64)
    costs = np.array([-5.0, -5.0, -5.0, 0.0, 0.0, 0.0, 0.0, 0.0], dtype=np.float32)
    sets[3] = 0
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    for S in range(1 << n):
        if S & 1:
            continue
        gc, gp = ulg_ctx.bestscore([0], [S])
        ec, ep = srch.bestscore(0, S)
        assert gc[0] == ec and int(gp[0]) == ep


def test_pattern_database_matches_oracle(ulg_ctx, oracle_built):
    o = oracle_built
    n = 13
    X, _ = synth.gaussian_sem(n, 1500, 9301)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 1.0, 3)
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    for pd_count in (1, 2, 3):
        srch.pdb_build(pd_count)
        ulg_ctx.pdb_build(pd_count)
        rng = np.random.default_rng(pd_count)
        Ss = _random_subsets(rng, n, 3000) + [0, (1 << n) - 1]
        h, comp = ulg_ctx.pdb_h(Ss)
        for S, hv, cv in zip(Ss, h, comp):
            eh, ec = srch.pdb_h(S)
            assert np.float32(hv).tobytes() == np.float32(eh).tobytes(), (pd_count, S)
            assert int(cv) == ec


@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", [0.5, 1.0, 2.0])
def test_gpu_pipeline_reproduces_golden_dag(ulg_ctx, oracle_built, fig, lam):
    """CSV -> GPU cBIC -> device "%f" round trip -> GPU tables/PDB -> exact A*
    reproduces triplet_data/Figure_*/astar_dag_*.csv, and the netFile text
    equals the oracle's."""
    X = load_fig(fig)
    n = X.shape[1]
    ulg_ctx.load(X, lam)
    ulg_ctx.score(list(range(n)), [(1 << n) - 1] * n, 3)
    ulg_ctx.search_from_scores()
    res = ulg_ctx.astar(edges=[(1 << n) - 1] * n, mode=0)
    M = oracle_built.dag_matrix(res["vpar"], n).tolist()
    assert M == fig_dag(fig)
    offs, sets, scores, costs = _oracle_pipeline(oracle_built, X, lam, 3)
    ref = oracle_built.Search(n, offs, sets, costs).astar(edges=[(1 << n) - 1] * n)
    assert res["net_text"] == ref["net_text"]
    assert res["expanded"] == ref["expanded"]
    assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()


@pytest.mark.parametrize("seed,n,k", [(9310, 10, 4), (9311, 13, 3), (9312, 15, 4), (9313, 16, 2)])
def test_exact_astar_matches_oracle(ulg_ctx, oracle_built, seed, n, k):
    o = oracle_built
    X, _ = synth.gaussian_sem(n, 3000, seed)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, k)
    ulg_ctx.search_load(offs, sets, costs)
    full = [(1 << n) - 1] * n
    res = ulg_ctx.astar(edges=full, mode=0)
    ref = o.Search(n, offs, sets, costs).astar(edges=full)
    assert ref["rc"] == 0
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert list(res["order"]) == list(ref["order"])
    assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
    assert res["expanded"] == ref["expanded"]
    # the GPU order-graph search finds the same optimal cost
    gres = ulg_ctx.astar(edges=full, mode=1)
    assert abs(gres["cost"] - ref["cost"]) <= 1e-6 * abs(ref["cost"])
    assert gres["expanded"] == (1 << n) - 1  # every node but the goal


def test_exact_astar_sparse_skeleton_components(ulg_ctx, oracle_built):
    """Two skeleton components plus the neighbour filter: the per-component
    rewrite of netFile/netFile.csv (astar_main.cpp:470,519) is reproduced."""
    import ulg
    o = oracle_built
    n = 14
    X1, W1 = synth.gaussian_sem(8, 2500, 9320)
    X2, W2 = synth.gaussian_sem(6, 2500, 9321)
    X = np.hstack([X1, X2])
    W = np.zeros((n, n))
    W[:8, :8] = W1
    W[8:, 8:] = W2
    rows = synth.true_skeleton_edges(W)
    cands = ulg.candidates_from_edges(rows, n)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, 3, cands)
    ulg_ctx.search_load(offs, sets, costs)
    res = ulg_ctx.astar(edges=rows, mode=0)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows)
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert res["net_text"] == ref["net_text"]
    assert res["expanded"] == ref["expanded"]


def test_c2_end_to_end_bit_exact(ulg_ctx, oracle_built):
    """BASELINE config C2 at full size (n=20, N=10k, k=4, full skeleton):
    GPU scoring + GPU tables + exact A* give the oracle's DAG bit for bit."""
    o = oracle_built
    n, N, k = 20, 10000, 4
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), full, k)
    ulg_ctx.search_from_scores()
    res = ulg_ctx.astar(edges=full, mode=0)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, k)
    ref = o.Search(n, offs, sets, costs).astar(edges=full)
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
    assert res["expanded"] == ref["expanded"]
    gres = ulg_ctx.astar(edges=full, mode=1)
    assert abs(gres["cost"] - ref["cost"]) <= 1e-6 * abs(ref["cost"])


@pytest.mark.parametrize("anc,scc", [(0b111, 0b111111111000), (0, 0b111111000000), (0b1, 0b110),
                                     (0b11110000, 0b1111)])
@pytest.mark.parametrize("sparse", [False, True])
def test_exact_astar_ancestors_and_scc(ulg_ctx, oracle_built, anc, scc, sparse):
    """astar -p/-s (astar_main.cpp:590-598,607): the pattern database over
    (ancestors, scc) and the per-component search started from the ancestors
    reproduce the oracle's DAG, cost, expansions and netFile text."""
    import ulg
    o = oracle_built
    n = 12
    X, W = synth.gaussian_sem(n, 3000, 9330)
    full = [(1 << n) - 1] * n
    rows = synth.true_skeleton_edges(W) if sparse else full
    cands = ulg.candidates_from_edges(rows, n) if sparse else None
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, 3, cands)
    ulg_ctx.search_load(offs, sets, costs)
    res = ulg_ctx.astar(edges=rows, mode=0, ancestors=anc, scc=scc)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows, ancestors=anc, scc=scc)
    assert ref["rc"] == 0
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
    assert res["expanded"] == ref["expanded"]
    assert res["net_text"] == ref["net_text"]
    # back to the whole lattice on the same context: the PDB is rebuilt
    res2 = ulg_ctx.astar(edges=rows, mode=0)
    ref2 = o.Search(n, offs, sets, costs).astar(edges=rows)
    assert [int(x) for x in res2["vpar"]] == [int(x) for x in ref2["vpar"]]
    assert res2["expanded"] == ref2["expanded"]


def test_gpu_mode_rejects_ancestors(ulg_ctx, oracle_built):
    o = oracle_built
    n = 8
    X, _ = synth.gaussian_sem(n, 1000, 9331)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, 2)
    ulg_ctx.search_load(offs, sets, costs)
    with pytest.raises(RuntimeError):
        ulg_ctx.astar(edges=[(1 << n) - 1] * n, mode=1, ancestors=0b1, scc=0b110)


@pytest.mark.parametrize("symmetric", [True, False])
def test_gpu_search_sparse_skeleton_optimal_cost(ulg_ctx, oracle_built, symmetric):
    """GPU layer search under the neighbour filter (astar_main.cpp:305-313):
    with symmetric rows it settles disconnected subsets without reading their
    predecessors; with asymmetric rows (a hand-edited skeleton file) it reads
    them all.  Either way the optimal cost equals the oracle's A*."""
    import ulg
    o = oracle_built
    n = 16
    X, W = synth.gaussian_sem(n, 3000, 9330)
    rows = synth.true_skeleton_edges(W, extra_frac=0.2, seed=5)
    if not symmetric:  # drop one direction of a few edges
        for i in range(n):
            nb = [j for j in range(n) if (rows[i] >> j) & 1 and j > i]
            if nb and i % 3 == 0:
                rows[i] &= ~(1 << nb[0])
    cands = ulg.candidates_from_edges(rows, n)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, 4, cands)
    ulg_ctx.search_load(offs, sets, costs)
    ulg_ctx.pdb_build(2)
    res = ulg_ctx.astar(edges=rows, mode=1, net_text=False)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows)
    assert ref["rc"] == 0
    assert abs(res["cost"] - ref["cost"]) <= 1e-6 * abs(ref["cost"]), (res["cost"], ref["cost"])


@pytest.mark.parametrize("sparse", [False, True])
def test_exact_astar_dense_and_indexed_forms_agree(ulg_ctx, oracle_built, monkeypatch, sparse):
    """Scopes of <= 26 variables run the dense replay (node homes at
    pext(S, scope), successor-cost rows); ULG_EXACT_SPARSE forces the
    indexed form used for larger scopes.  Both give the oracle's DAG, order,
    cost and expansion count, on a full skeleton and on a sparse one."""
    import ulg
    o = oracle_built
    n, k = 18, 4
    X, W = synth.gaussian_sem(n, 4000, 9350)
    rows = synth.true_skeleton_edges(W, extra_frac=0.5, seed=4) if sparse else [(1 << n) - 1] * n
    cands = ulg.candidates_from_edges(rows, n)
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, k, cands)
    ulg_ctx.search_load(offs, sets, costs)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows)
    out = []
    for force in (False, True):
        if force:
            monkeypatch.setenv("ULG_EXACT_SPARSE", "1")
        else:
            monkeypatch.delenv("ULG_EXACT_SPARSE", raising=False)
        res = ulg_ctx.astar(edges=rows, mode=0)
        assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
        assert list(res["order"]) == list(ref["order"])
        assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
        assert res["expanded"] == ref["expanded"]
        assert res["net_text"] == ref["net_text"]
        out.append(res["expanded"])
    assert out[0] == out[1]


@pytest.mark.parametrize("pf", ["0", "2", "4", "260", "772"])
def test_exact_astar_prefetch_modes_identical(ulg_ctx, oracle_built, monkeypatch, pf):
    """ULG_EXACT_PF only moves prefetches (bit 1: five heap levels ahead in a
    pop; bit 2: the heap top's records and cost row before its pop) or, with
    value 256, the heap's physical layout (PairBlockLayout, exact_heap.h;
    512: its deeper prefetch): the dense replay's DAG, order, cost and
    expansion count stay the oracle's in every mode."""
    import ulg
    o = oracle_built
    n, k = 18, 4
    X, _ = synth.gaussian_sem(n, 4000, 9351)
    rows = [(1 << n) - 1] * n
    offs, sets, scores, costs = _oracle_pipeline(o, X, 2.0, k, ulg.candidates_from_edges(rows, n))
    ulg_ctx.search_load(offs, sets, costs)
    ref = o.Search(n, offs, sets, costs).astar(edges=rows)
    monkeypatch.setenv("ULG_EXACT_PF", pf)
    res = ulg_ctx.astar(edges=rows, mode=0)
    assert [int(x) for x in res["vpar"]] == [int(x) for x in ref["vpar"]]
    assert list(res["order"]) == list(ref["order"])
    assert np.float32(res["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
    assert res["expanded"] == ref["expanded"]
