"""GPU parity tests of the cBIC scorer (libulg.so on cuda:0) against the CPU
oracle.  Bar: the stored parent-set lists are identical (index work,
bit-exact); scores agree within 1e-6 relative (north_star tolerance; the
oracle solves each OLS over all N rows, the GPU through the Gram matrix)."""
import math

import numpy as np
import pytest

from conftest import load_fig
import synth

pytestmark = pytest.mark.gpu

REL_TOL = 1e-6
DEFAULT_VARIANT = 241  # the library default (ulg_internal.h)


def _compare_lists(o_offs, o_sets, o_scores, g_offs, g_sets, g_scores, variables, ctx=""):
    assert len(o_offs) == len(g_offs), ctx
    for i, v in enumerate(variables):
        a = o_sets[o_offs[i]:o_offs[i + 1]]
        b = g_sets[g_offs[i]:g_offs[i + 1]]
        if not np.array_equal(a, b):
            sa, sb = set(int(x) for x in a), set(int(x) for x in b)
            raise AssertionError(f"{ctx} variable {v}: stored sets differ: only oracle {sorted(sa - sb)[:8]}, "
                                 f"only gpu {sorted(sb - sa)[:8]} ({len(a)} vs {len(b)})")
        sa = o_scores[o_offs[i]:o_offs[i + 1]].astype(np.float64)
        sb = g_scores[g_offs[i]:g_offs[i + 1]].astype(np.float64)
        err = np.abs(sa - sb) / np.maximum(np.abs(sa), 1.0)
        assert err.max(initial=0.0) <= REL_TOL, f"{ctx} variable {v}: max rel score error {err.max()}"


def _oracle_lists(oracle, X, lam, variables, cands, k):
    ds = oracle.Dataset(X)
    offs = [0]
    sets, scores = [], []
    for v, c in zip(variables, cands):
        s, sc = ds.score_variable(lam, v, c, k)
        sets.append(s)
        scores.append(sc)
        offs.append(offs[-1] + len(s))
    return np.array(offs), np.concatenate(sets), np.concatenate(scores)


def test_gram_matches_numpy(ulg_ctx):
    X, _ = synth.gaussian_sem(21, 7000, 9100)
    ulg_ctx.load(X, 2.0)
    G = ulg_ctx.gram()
    Z = (X - X.mean(0)) / X.std(0, ddof=1)
    ref = Z.T @ Z
    assert np.allclose(G, ref, rtol=1e-11, atol=1e-8 * len(X))
    # asymmetric check: individual off-diagonal entries, not just symmetry
    assert abs(G[3, 17] - ref[3, 17]) <= 1e-9 * len(X)
    assert np.allclose(G, G.T, rtol=0, atol=1e-9 * len(X))


@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", [0.5, 1.0, 2.0])
def test_fig_scores_match_oracle(ulg_ctx, oracle_built, fig, lam):
    X = load_fig(fig)
    n = X.shape[1]
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, lam)
    g = ulg_ctx.score_all(variables, cands, 3)
    o = _oracle_lists(oracle_built, X, lam, variables, cands, 3)
    _compare_lists(*o, *g, variables, ctx=f"fig{fig} lam={lam}")


@pytest.mark.parametrize("seed,n,N,k", [(9200, 10, 3000, 4), (9201, 12, 2000, 6), (9202, 9, 1500, 8),
                                        (9203, 14, 1000, 3), (9204, 8, 800, 7)])
def test_synthetic_full_skeleton_matches_oracle(ulg_ctx, oracle_built, seed, n, N, k):
    X, _ = synth.gaussian_sem(n, N, seed)
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    g = ulg_ctx.score_all(variables, cands, k)
    o = _oracle_lists(oracle_built, X, 2.0, variables, cands, k)
    _compare_lists(*o, *g, variables, ctx=f"seed {seed}")


def test_sparse_skeleton_and_variable_subset(ulg_ctx, oracle_built):
    """2-hop candidate sets from a sparse skeleton; a permuted subset of the
    variables; variable 0 both inside and outside the candidate lists."""
    import ulg
    n = 16
    X, W = synth.gaussian_sem(n, 2500, 9210)
    rows = synth.true_skeleton_edges(W, extra_frac=0.1, seed=3)
    cands_all = ulg.candidates_from_edges(rows, n)
    variables = [7, 0, 13, 2, 9]
    cands = [cands_all[v] for v in variables]
    ulg_ctx.load(X, 1.0)
    g = ulg_ctx.score_all(variables, cands, 4)
    o = _oracle_lists(oracle_built, X, 1.0, variables, cands, 4)
    _compare_lists(*o, *g, variables, ctx="sparse")


@pytest.mark.parametrize("k", [0, 1, 9, 12])
def test_edge_parent_limits_and_isolated_variables(ulg_ctx, oracle_built, k):
    """Edge cases of calculateScores_internal (score_calculator.cpp:54-135):
    -p 0 (no limit: n - 1, score_main.cpp:296-298), a limit above the
    candidate count (layers stop at m), a variable whose candidate set is
    itself only (m = 0), one whose only candidate is variable 0, and a
    skeleton row without variable 0."""
    n = 12
    X, _ = synth.gaussian_sem(n, 900, 9220)
    full = (1 << n) - 1
    variables = [0, 3, 5, 7, 11, 1]
    cands = [full, 1 << 3, (1 << 5) | 1, full & ~1, (1 << 11) | (1 << 4) | (1 << 9), full]
    ulg_ctx.load(X, 2.0)
    g = ulg_ctx.score_all(variables, cands, k)
    o = _oracle_lists(oracle_built, X, 2.0, variables, cands, k if k >= 1 else n - 1)
    _compare_lists(*o, *g, variables, ctx=f"edge k={k}")
    assert g[0][variables.index(3) + 1] - g[0][variables.index(3)] == 1  # m = 0: the empty set alone


def test_constant_column_nan_scores_match_oracle(ulg_ctx, oracle_built):
    """A constant column normalises to NaN (x - mean = 0, sd = 0, as
    BIC_OLS.cpp:66-97 divides): every set containing it, and the variable's
    own sets, score NaN.  NaN is never >= -ts and never pruned, so such sets
    are stored and stop the subset recursion like any stored key; the absent
    sentinel (a NaN of its own payload) must not swallow them."""
    n = 7
    X, _ = synth.gaussian_sem(n, 600, 9230)
    X[:, 2] = 3.0
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    g_offs, g_sets, g_sc = ulg_ctx.score_all(variables, cands, 4)
    o_offs, o_sets, o_sc = _oracle_lists(oracle_built, X, 2.0, variables, cands, 4)
    assert np.array_equal(o_offs, g_offs) and np.array_equal(o_sets, g_sets)
    assert np.array_equal(np.isnan(o_sc), np.isnan(g_sc)) and np.isnan(g_sc).any()
    ok = ~np.isnan(o_sc)
    err = np.abs(o_sc[ok].astype(np.float64) - g_sc[ok]) / np.maximum(np.abs(o_sc[ok]), 1.0)
    assert err.max(initial=0.0) <= REL_TOL


def test_parent_limit_above_gpu_maximum_fails_loudly(ulg_ctx):
    """More than ULG_MAX_PARENTS_GPU (31) parents: a status code and a
    message, not a silent truncation."""
    import ulg
    n = 40
    X, _ = synth.gaussian_sem(n, 200, 9221)
    ulg_ctx.load(X, 2.0)
    with pytest.raises(ulg.ULGError, match="ULG_MAX_PARENTS_GPU"):
        ulg_ctx.score([0], [(1 << n) - 1], 32)


def test_quantize_matches_oracle(ulg_ctx, oracle_built):
    rng = np.random.default_rng(7)
    vals = np.concatenate([rng.normal(0, 3e4, 20000), rng.normal(0, 1, 20000), rng.normal(0, 1e-5, 5000),
                           [0.0078125, 0.0234375, -0.0078125, -1e-9, 1e-9, 0.0, -0.0, 5e-7, -5e-7, 3e38, -3e38,
                            1e-40, np.inf, -np.inf]]).astype(np.float32)
    got = ulg_ctx.quantize(vals)
    exp = np.array([oracle_built.quantize(float(x)) for x in vals], dtype=np.float32)
    assert got.tobytes() == exp.tobytes()


def test_c2_properties_full_size(ulg_ctx, oracle_built):
    """BASELINE config C2 (n=20, N=10k, k=4, full skeleton) at full size:
    size-independent properties on every variable, oracle parity on two."""
    n, N, k = 20, 10000, 4
    X, _ = synth.gaussian_sem(n, N, 9200)
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    stored, scored = ulg_ctx.score(variables, cands, k)
    assert scored == n * sum(math.comb(n - 1, L) for L in range(k + 1)) == 100720
    offs, sets, scores = ulg_ctx.fetch(stored)
    assert offs[0] == 0 and offs[-1] == stored
    for v in range(n):
        s = sets[offs[v]:offs[v + 1]]
        assert int(s[0]) == 0 and np.float32(scores[offs[v]]).tobytes() == np.float32(-0.0).tobytes()
        keys = [(bin(int(x)).count("1"), int(x)) for x in s]
        assert keys == sorted(keys) and len(set(keys)) == len(keys)
        assert all(not ((int(x) >> v) & 1) and bin(int(x)).count("1") <= k for x in s)
    assert np.isfinite(scores).all()
    for v in (0, 11):
        o = _oracle_lists(oracle_built, X, 2.0, [v], [cands[v]], k)
        g = (np.array([0, offs[v + 1] - offs[v]]), sets[offs[v]:offs[v + 1]], scores[offs[v]:offs[v + 1]])
        _compare_lists(*o, *g, [v], ctx="C2")


def test_rescoring_is_deterministic(ulg_ctx):
    X, _ = synth.gaussian_sem(15, 4000, 9220)
    ulg_ctx.load(X, 2.0)
    a = ulg_ctx.score_all(list(range(15)), [(1 << 15) - 1] * 15, 5)
    b = ulg_ctx.score_all(list(range(15)), [(1 << 15) - 1] * 15, 5)
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()


@pytest.mark.parametrize("variant", [1, 49, 65, 113, 241])
def test_scorer_variants_identical(ulg_ctx, oracle_built, variant):
    """Every scorer variant (presence gather x recursion form x decision-only
    walk x subset-maxima settling) stores exactly the oracle's sets (k=6
    exercises the unrolled presence, k=7,8 the loop)."""
    n = 11
    X, _ = synth.gaussian_sem(n, 2500, 9230 + variant)
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.set_option("score_variant", variant)
    try:
        for k in (6, 8):
            g = ulg_ctx.score_all(variables, cands, k)
            o = _oracle_lists(oracle_built, X, 2.0, variables, cands, k)
            _compare_lists(*o, *g, variables, ctx=f"variant {variant} k={k}")
    finally:
        ulg_ctx.set_option("score_variant", DEFAULT_VARIANT)


@pytest.mark.parametrize("sets_per_lane", ["1", "2", "4", "8"])
def test_walk_forms_identical(ulg_ctx, oracle_built, monkeypatch, sets_per_lane):
    """The bit-sliced walk with 1, 2, 4 or 8 sets per lane (ULG_SLICED_K) stores
    exactly the oracle's sets, with and without variable 0 among the
    candidates (both N4 phases)."""
    monkeypatch.setenv("ULG_SLICED_K", sets_per_lane)
    n = 12
    X, _ = synth.gaussian_sem(n, 3000, 9250)
    ulg_ctx.load(X, 2.0)
    for cands in ([(1 << n) - 1] * n, [((1 << n) - 1) & ~1] * n):
        variables = list(range(1, n)) if cands[0] & 1 == 0 else list(range(n))
        cands = cands[:len(variables)]
        g = ulg_ctx.score_all(variables, cands, 6)
        o = _oracle_lists(oracle_built, X, 2.0, variables, cands, 6)
        _compare_lists(*o, *g, variables, ctx=f"ULG_SLICED_K={sets_per_lane}")


def test_subset_maxima_identical_c3_and_without_var0(ulg_ctx):
    """Variants 113 (subset maxima settle sets before the presence gathers,
    the rule keys gathered before the rest) and 241 (113 with the sets the
    rules leave to the walk compacted a second time) against 49 (every set
    gathered in full): identical lists at C3 and on candidate
    lists without variable 0 (phase 1 then has no P\\a+{0} keys)."""
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    ulg_ctx.load(X, 2.0)
    cases = [(list(range(n)), [(1 << n) - 1] * n, 6), (list(range(1, n)), [((1 << n) - 1) & ~1] * (n - 1), 6),
             (list(range(n)), [((1 << n) - 1) & ~(1 << (v % 5)) for v in range(n)], 7)]
    try:
        for variables, cands, k in cases:
            res = {}
            for variant in (49, 113, 241):
                ulg_ctx.set_option("score_variant", variant)
                res[variant] = ulg_ctx.score_all(variables, cands, k)
            for other in (113, 241):
                for a, b in zip(res[49], res[other]):
                    assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (len(variables), k, other)
    finally:
        ulg_ctx.set_option("score_variant", DEFAULT_VARIANT)


def test_walk_forms_identical_c3(ulg_ctx, monkeypatch):
    """At C3 (n=25, N=10k, k=6, full skeleton: 4,751,275 sets) 2 and 8 sets
    per lane store the default walk's lists bit for bit."""
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    ulg_ctx.load(X, 2.0)
    res = {}
    for k in ("4", "2", "8"):
        monkeypatch.setenv("ULG_SLICED_K", k)
        res[k] = ulg_ctx.score_all(list(range(n)), [(1 << n) - 1] * n, 6)
    for k in ("2", "8"):
        for a, b in zip(res["4"], res[k]):
            assert a.tobytes() == b.tobytes(), k


def test_walk_k6_option_identical_c3_and_segments(ulg_ctx):
    """ulg_set_option("walk_k6"): 1, 2 and 8 sets per lane in the layer-6
    walks store the default's (4) lists bit for bit at C3, with one stream
    group (one walk-queue segment set per launch) and three (every group's
    segment counters at their own offsets)."""
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    ulg_ctx.load(X, 2.0)
    full = [(1 << n) - 1] * n
    try:
        for streams in (1, 3):
            ulg_ctx.set_option("score_streams", streams)
            ulg_ctx.set_option("walk_k6", 4)
            ref = ulg_ctx.score_all(list(range(n)), full, 6)
            for k6 in (1, 2, 8):
                ulg_ctx.set_option("walk_k6", k6)
                got = ulg_ctx.score_all(list(range(n)), full, 6)
                for a, b in zip(ref, got):
                    assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (streams, k6)
    finally:
        ulg_ctx.set_option("walk_k6", 4)
        ulg_ctx.set_option("score_streams", 3)


@pytest.mark.parametrize("option", ["walk_bucket"])
@pytest.mark.parametrize("variant", [113, 241])
def test_walk_forms_match_oracle(ulg_ctx, oracle_built, variant, option):
    """ulg_set_option("walk_bucket", 0 / 1): the layer-5/6 queues walked in
    queue order (walk_sliced_kernel) or sorted by walk key
    (walk_bucket_kernel) -- the oracle's sets with and without variable 0
    among the candidates (both N4 phases), k = 6, and on a sparse
    skeleton."""
    n = 12
    X, _ = synth.gaussian_sem(n, 3000, 9251)
    ulg_ctx.load(X, 2.0)
    rng = np.random.default_rng(5)
    sparse = [int(((1 << n) - 1) & ~int(rng.integers(0, 1 << n))) | 1 for _ in range(n)]
    try:
        ulg_ctx.set_option("score_variant", variant)
        ulg_ctx.set_option(option, 1)
        for cands in ([(1 << n) - 1] * n, [((1 << n) - 1) & ~1] * n, sparse):
            variables = list(range(1, n)) if cands[0] & 1 == 0 else list(range(n))
            cands = cands[:len(variables)]
            g = ulg_ctx.score_all(variables, cands, 6)
            assert ulg_ctx.info("score_error_word") == 0
            o = _oracle_lists(oracle_built, X, 2.0, variables, cands, 6)
            _compare_lists(*o, *g, variables, ctx=f"{option} variant {variant}")
    finally:
        ulg_ctx.set_option(option, 0)
        ulg_ctx.set_option("score_variant", DEFAULT_VARIANT)


@pytest.mark.parametrize("option", ["walk_bucket"])
def test_walk_forms_identical_c3_c5(ulg_ctx, option):
    """The key-sorted walk stores the queue-order walk's lists bit for bit at C3 (and so the oracle command lines',
    tests/golden/c3_oracle.json) and at the k = 6 C5 shape, with one and
    three stream groups, 4 and 8 sets per lane at layer 6 (walk_k6)."""
    for n, N in ((25, 10000), (32, 50000)):
        X, _ = synth.gaussian_sem(n, N, 9200)
        ulg_ctx.load(X, 2.0)
        full = [(1 << n) - 1] * n
        try:
            for streams, k6 in ((1, 4), (3, 4), (1, 8)):
                ulg_ctx.set_option("score_streams", streams)
                ulg_ctx.set_option("walk_k6", k6)
                ulg_ctx.set_option(option, 0)
                ref = ulg_ctx.score_all(list(range(n)), full, 6)
                ulg_ctx.set_option(option, 1)
                got = ulg_ctx.score_all(list(range(n)), full, 6)
                assert ulg_ctx.info("score_error_word") == 0
                for a, b in zip(ref, got):
                    assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (n, streams, k6)
        finally:
            ulg_ctx.set_option(option, 0)
            ulg_ctx.set_option("walk_k6", 4)
            ulg_ctx.set_option("score_streams", 3)


def test_score_fused_small_layers_identical(ulg_ctx):
    """ulg_set_option("score_fused"): layers up to 1..4 in one launch (a
    workgroup per variable, its layers and phases in order) store the
    per-layer launches' lists bit for bit: C3 (k = 6, the layers above the
    fused ones read its subset maxima), a call whose top layer is fused
    (k = 3: no layer reads layer 3's phase-1 maxima), a sparse candidate
    set, and variables without variable 0 among their candidates."""
    rng = np.random.default_rng(31)
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    ulg_ctx.load(X, 2.0)
    full = [(1 << n) - 1] * n
    sparse = [int(rng.integers(1, 1 << n)) | (1 << int(rng.integers(0, n))) for _ in range(n)]
    no0 = [((1 << n) - 1) & ~1] * n
    try:
        for cands, k in ((full, 6), (full, 3), (sparse, 6), (no0, 5)):
            ulg_ctx.set_option("score_fused", 0)
            ref = ulg_ctx.score_all(list(range(n)), cands, k)
            for f in (1, 2, 3, 4):
                ulg_ctx.set_option("score_fused", f)
                got = ulg_ctx.score_all(list(range(n)), cands, k)
                for a, b in zip(ref, got):
                    assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (k, f)
    finally:
        ulg_ctx.set_option("score_fused", 3)


def test_score_graph_replay_identical_and_profiled(ulg_ctx):
    """ulg_set_option("score_graph"): the scoring launch sequence is captured
    into a hipGraph on the first call and replayed on the next ones with the
    same variables, limits and buffers.  The lists are identical with and
    without it, across replays, after a reload with other data and another
    lambda (same shapes: the graph replays with the new Gram matrix and the
    recapture picks up the new lambda), and a call with other variables
    recaptures.  With profiling on the calls run unrolled (HIP events time
    every kernel)."""
    n, N, k = 20, 10000, 4
    outs = []
    try:
        for graph in (0, 1, 1, 1):
            ulg_ctx.set_option("score_graph", graph)
            X, _ = synth.gaussian_sem(n, N, 9200)
            ulg_ctx.load(X, 2.0)
            outs.append(ulg_ctx.score_all(list(range(n)), [(1 << n) - 1] * n, k))
        # other data, other lambda, then a variable subset (recapture)
        res = {}
        for graph in (0, 1):
            ulg_ctx.set_option("score_graph", graph)
            X2, _ = synth.gaussian_sem(n, N, 9201)
            ulg_ctx.load(X2, 1.0)
            a = ulg_ctx.score_all(list(range(n)), [(1 << n) - 1] * n, k)
            b = ulg_ctx.score_all([3, 7, 11], [(1 << n) - 1] * 3, k)
            res[graph] = (a, b)
        ulg_ctx.set_option("score_graph", 1)
        ulg_ctx.profile(True)
        ulg_ctx.profile_select(["score_layer_4_rest"])
        ulg_ctx.profile_reset()
        for _ in range(3):
            ulg_ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
        p = ulg_ctx.profile_get("score_layer_4_rest")
    finally:
        ulg_ctx.profile(False)
        ulg_ctx.profile_select(None)
        ulg_ctx.set_option("score_graph", 1)
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes()
    for x, y in zip(res[0][0] + res[0][1], res[1][0] + res[1][1]):
        assert np.asarray(x).tobytes() == np.asarray(y).tobytes()
    assert p is not None and p["count"] == 3 and p["avg_ms"] > 0
