"""GPU parity tests of ulg_triplet_astar (astar/triplet_astar.cpp:285-1622):
the MEC matrix, the number of A* runs, the distinct clusters searched and the
total expansions equal the oracle's restatement (tests/test_oracle_golden.py
pins that against both triplet_mec fixtures), and the full GPU pipeline
reproduces the fixtures themselves."""
import numpy as np
import pytest

from conftest import TRIPLET_SKELETON, fig_mec, load_fig
import synth
import ulg

pytestmark = pytest.mark.gpu


def _skeleton_rows(text):
    return [sum(int(x) << j for j, x in enumerate(line.split(","))) for line in text.strip().splitlines()]


def _oracle_costs(o, X, lam, k, cands):
    ds = o.Dataset(X)
    offs, sets, scores = ds.score_all(lam, cands, k, threads=8)
    costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
    return offs, sets, costs


@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", [0.5, 1.0, 2.0])
def test_gpu_pipeline_reproduces_triplet_mec(ulg_ctx, oracle_built, fig, lam):
    """CSV -> GPU cBIC -> device "%f" round trip -> GPU tables -> triplet driver."""
    X = load_fig(fig)
    n = X.shape[1]
    rows = _skeleton_rows(TRIPLET_SKELETON[fig])
    ulg_ctx.load(X, lam)
    ulg_ctx.score(list(range(n)), ulg.candidates_from_edges(rows, n), 3)
    ulg_ctx.search_from_scores()
    res = ulg_ctx.triplet(edges=rows)
    assert res["mec"].tolist() == fig_mec(fig)
    offs, sets, costs = _oracle_costs(oracle_built, X, lam, 3, ulg.candidates_from_edges(rows, n))
    ref = oracle_built.triplet(oracle_built.Search(n, offs, sets, costs), edges=rows)
    assert (res["runs"], res["distinct"], res["expanded"]) == (ref["runs"], ref["distinct"], ref["expanded"])


@pytest.mark.parametrize("seed,n,extra,k,diag", [
    (9400, 8, 0.0, 3, True), (9401, 10, 0.1, 3, True), (9402, 12, 0.05, 4, True), (9403, 14, 0.1, 3, True),
    (9401, 10, 0.1, 3, False), (9402, 12, 0.05, 4, False), (9403, 14, 0.1, 3, False), (9405, 16, 0.05, 3, False),
])
def test_triplet_matches_oracle_sparse(ulg_ctx, oracle_built, seed, n, extra, k, diag):
    """Sparse skeletons (true edges + a fraction of spurious ones), with and
    without the diagonal: many distinct clusters, v-structures, unfaithful
    edges and Meek orientations."""
    o = oracle_built
    X, W = synth.gaussian_sem(n, 3000, seed)
    rows = synth.true_skeleton_edges(W, extra, seed)
    if not diag:
        rows = [r & ~(1 << i) for i, r in enumerate(rows)]
    offs, sets, costs = _oracle_costs(o, X, 2.0, k, ulg.candidates_from_edges(rows, n))
    ulg_ctx.search_load(offs, sets, costs)
    res = ulg_ctx.triplet(edges=rows)
    ref = o.triplet(o.Search(n, offs, sets, costs), edges=rows)
    assert ref["rc"] == 0
    assert res["mec"].tolist() == ref["mec"].tolist()
    assert (res["runs"], res["distinct"], res["expanded"]) == (ref["runs"], ref["distinct"], ref["expanded"])


@pytest.mark.parametrize("skeleton", ["none", "offdiag"])
def test_triplet_full_skeleton_one_cluster(ulg_ctx, oracle_built, skeleton):
    """No skeleton (every row is the full set, self included) or the full
    off-diagonal skeleton: every triple's cluster is all n variables, so one
    search serves every run."""
    o = oracle_built
    n = 11
    X, _ = synth.gaussian_sem(n, 3000, 9406)
    full = [(1 << n) - 1] * n
    offs, sets, costs = _oracle_costs(o, X, 1.0, 3, full)
    ulg_ctx.search_load(offs, sets, costs)
    rows = None if skeleton == "none" else [((1 << n) - 1) & ~(1 << i) for i in range(n)]
    res = ulg_ctx.triplet(edges=rows)
    ref = o.triplet(o.Search(n, offs, sets, costs), edges=rows)
    assert res["distinct"] == 1 and res["runs"] == ref["runs"]
    assert res["mec"].tolist() == ref["mec"].tolist()
    assert res["expanded"] == ref["expanded"]


def test_cluster_pattern_databases_match_oracle(ulg_ctx, oracle_built):
    """StaticPatternDatabase over a cluster (ancestors, scc) as triplet_astar
    builds it per run (triplet_astar.cpp:303): every h the search can ask."""
    o = oracle_built
    n = 12
    X, _ = synth.gaussian_sem(n, 2000, 9407)
    full = [(1 << n) - 1] * n
    offs, sets, costs = _oracle_costs(o, X, 2.0, 3, full)
    ulg_ctx.search_load(offs, sets, costs)
    srch = o.Search(n, offs, sets, costs)
    rng = np.random.default_rng(7)
    for scc, anc, pd in [(0b000011110110, 0, 2), (0b101010101011, 0, 3), (0b000000000111, 0, 1),
                         (0b011100111000, 0b100000000001, 2)]:
        srch.pdb_build(pd, anc, scc)
        ulg_ctx.pdb_build(pd, anc, scc)
        Ss = [int(x) & scc for x in rng.integers(0, 1 << n, 500, dtype=np.int64)] + [0, scc]
        h, comp = ulg_ctx.pdb_h(Ss)
        for S, hv, cv in zip(Ss, h, comp):
            eh, ec = srch.pdb_h(S)
            assert np.float32(hv).tobytes() == np.float32(eh).tobytes(), (scc, S)
            assert int(cv) == ec
