"""ulg_cbic_score_async / ulg_cbic_score_finish: a scoring call queued
without waiting gives the lists ulg_cbic_score gives, also with two
contexts' calls in flight at once on one GPU (the throughput loop of
scripts/slots_probe.py), and a later scorer call or fetch collects a
pending one first."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _lists(ctx, stored):
    offs, sets, scores = ctx.fetch(stored)
    return np.asarray(offs).copy(), np.asarray(sets).copy(), np.asarray(scores).copy()


@pytest.mark.parametrize("n,k", [(20, 4), (25, 6)])
def test_async_scoring_equals_sync(n, k):
    import ulg
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    full = [(1 << n) - 1] * n
    a, b = ulg.Context(0), ulg.Context(0)
    try:
        for c in (a, b):
            c.load(X, 2.0)
        st, sc = a.score(list(range(n)), full, k)
        ref = _lists(a, st)
        half = list(range(0, n, 2))
        st_h, _ = a.score(half, [full[v] for v in half], k)
        ref_h = _lists(a, st_h)
        for _ in range(3):
            # two calls in flight on two contexts, finished in launch order
            a.score_async(list(range(n)), full, k)
            b.score_async(half, [full[v] for v in half], k)
            assert a.score_finish() == (st, sc)
            sb, _ = b.score_finish()
            assert sb == st_h
            for got, want in ((_lists(a, st), ref), (_lists(b, sb), ref_h)):
                assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
                assert got[2].tobytes() == want[2].tobytes()
        # a pending call is collected by the next call / fetch on its context
        a.score_async(list(range(n)), full, k)
        got = _lists(a, st)
        assert np.array_equal(got[1], ref[1]) and got[2].tobytes() == ref[2].tobytes()
        a.score_async(half, [full[v] for v in half], k)
        assert a.score(list(range(n)), full, k) == (st, sc)
    finally:
        a.close()
        b.close()
