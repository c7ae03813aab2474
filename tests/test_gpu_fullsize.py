"""Parity at BASELINE.json's full sizes through a size-independent property:
the oracle cannot score C3's 4.75 M sets in test time, but it can re-decide
any single set under the reference's rule (BIC_OLS.cpp:174-276 with the
find_best_subset_score replay) against the cache the GPU run left behind.
Every sampled set must be stored exactly when the GPU stored it, with the
score within 1e-6 relative."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [("c3", 25, 10000, 6)])
def test_full_size_store_decisions(ulg_ctx, oracle_built, cfg):
    name, n, N, k = cfg
    o = oracle_built
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), full, k)
    ds = o.Dataset(X)
    rng = np.random.default_rng(17)
    checked = stored_hits = 0
    for v in (0, 7, 24):
        s_v = sets[offs[v]:offs[v + 1]]
        f_v = scores[offs[v]:offs[v + 1]]
        cache = o.Cache(s_v, f_v)
        gpu = {int(s): np.float32(f) for s, f in zip(s_v, f_v)}
        others = [u for u in range(n) if u != v]
        # random sets of every layer, both phases, plus stored ones
        picks = []
        for L in range(1, k + 1):
            for _ in range(40):
                picks.append(sum(1 << int(u) for u in rng.choice(others, size=L, replace=False)))
        picks += [int(x) for x in rng.choice(s_v, size=min(120, len(s_v)), replace=False)]
        for P in picks:
            st, val = ds.decide(2.0, v, P, cache)
            assert st == (P in gpu), (name, v, P, val)
            if st:
                g = float(gpu[P])
                assert abs(g - val) <= 1e-6 * max(abs(val), 1e-30), (v, P, g, val)
                stored_hits += 1
            checked += 1
    assert checked > 800 and stored_hits > 300
