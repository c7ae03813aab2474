"""ulg_cbic_score_sets: the per-call counterpart of
ScoringFunction::calculateScore (scoring_function.h:16-23, BIC_OLS.cpp:174-276).
Its value for a stored set must be the score ulg_cbic_score stored for it (same
Cholesky, bit for bit), agree with the oracle's per-row OLS within the scorer's
1e-6 relative tolerance for any set (including wide ones the layer scorer only
reaches past layer 8), and follow the reference on an empty parent set
(calculateScoreAndBeta returns 0, BIC_OLS.cpp:300-303) and on the variable's own
bit (parent_vec skips it)."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

REL_TOL = 1e-6


def test_score_sets_equal_stored_scores(ulg_ctx):
    n, N, k = 20, 10000, 4
    X, _ = synth.gaussian_sem(n, N, 9100)
    ulg_ctx.load(X, 2.0)
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), [(1 << n) - 1] * n, k)
    vars_ = np.repeat(np.arange(n, dtype=np.int32), np.diff(offs))
    got = ulg_ctx.score_sets(vars_, sets)
    nonempty = sets != 0
    assert nonempty.sum() > 1000
    assert np.array_equal(got[nonempty].view(np.uint32), scores[nonempty].view(np.uint32))
    # the empty set: the reference's calculateScore returns -0.0
    assert np.all(got[~nonempty] == 0.0) and np.all(np.signbit(got[~nonempty]))


def test_score_sets_match_oracle_and_ignore_own_bit(ulg_ctx, oracle_built):
    n, N = 30, 20000
    X, _ = synth.gaussian_sem(n, N, 9300)
    lam = 0.5
    ulg_ctx.load(X, lam)
    ds = oracle_built.Dataset(X)
    rng = np.random.default_rng(7)
    vars_, parents = [], []
    for _ in range(400):
        v = int(rng.integers(n))
        size = int(rng.integers(0, 25))
        others = [x for x in range(n) if x != v]
        P = 0
        for b in rng.choice(others, size=size, replace=False):
            P |= 1 << int(b)
        vars_.append(v)
        parents.append(P)
    got = ulg_ctx.score_sets(vars_, parents)
    # the variable's own bit is ignored
    got_own = ulg_ctx.score_sets(vars_, [p | (1 << v) for v, p in zip(vars_, parents)])
    assert np.array_equal(got.view(np.uint32), got_own.view(np.uint32))
    for v, P, g in zip(vars_, parents, got):
        ref = -float(ds.cbic_raw(lam, v, P))
        assert abs(float(g) - ref) <= REL_TOL * max(abs(ref), 1.0), (v, hex(P), float(g), ref)


def test_score_sets_rejects_bad_input(ulg_ctx):
    import ulg
    n, N = 8, 2000
    X, _ = synth.gaussian_sem(n, N, 9400)
    ulg_ctx.load(X, 2.0)
    with pytest.raises(ulg.ULGError):
        ulg_ctx.score_sets([n], [1])
    with pytest.raises(ulg.ULGError):
        ulg_ctx.score_sets([0], [1 << n])
    assert len(ulg_ctx.score_sets([], [])) == 0
