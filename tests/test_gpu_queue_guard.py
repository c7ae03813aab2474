"""The walk queue's device-side guards (round 6).

A scoring call's error word (ulg_get_info "score_error_word") gets bit 1
when a lane's walk-queue position falls past its segment (queue_walk then
writes nothing) and bit 2 when a walk entry names a slot past the call's
table (walk_store then writes nothing); either makes the call return a
nonzero status.  Round 5 faulted the GPU once on exactly these shapes (the
first "small" case of scripts/score_probe.py, three stream groups) while the
segmented queue was being written.  Here the word must stay 0 on those shapes
with one and three stream groups, synchronous and asynchronous, and the lists
must equal the oracle's."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

# scripts/score_probe.py CASES["small"]: (n, N, k, candidate kind)
SMALL = [(11, 2500, 6, "full"), (12, 3000, 6, "novar0"), (9, 2000, 4, "full"), (14, 3000, 5, "sparse")]


def _cands(n, kind, seed):
    full = (1 << n) - 1
    if kind == "full":
        return list(range(n)), [full] * n
    if kind == "novar0":
        return list(range(1, n)), [full & ~1] * (n - 1)
    rng = np.random.default_rng(seed)
    return list(range(n)), [int(full & ~int(rng.integers(0, 1 << n))) | 1 for _ in range(n)]


@pytest.mark.parametrize("n,N,k,kind", SMALL)
def test_error_word_stays_zero_small_shapes(oracle_built, n, N, k, kind):
    import ulg
    X, _ = synth.gaussian_sem(n, N, 9200)
    variables, cands = _cands(n, kind, n)
    ds = oracle_built.Dataset(X)
    ref = [ds.score_variable(2.0, v, c, k)[0] for v, c in zip(variables, cands)]
    for streams in (1, 3):
        ctx = ulg.Context(0)
        try:
            ctx.set_option("score_streams", streams)
            ctx.load(X, 2.0)
            for mode in ("sync", "sync", "async"):  # the second call replays the captured graph
                if mode == "async":
                    ctx.score_async(variables, cands, k)
                    st, _ = ctx.score_finish()
                else:
                    st, _ = ctx.score(variables, cands, k)
                assert ctx.info("score_error_word") == 0, (streams, mode)
                offs, sets, _ = ctx.fetch(st)
                for i, v in enumerate(variables):
                    assert np.array_equal(sets[offs[i]:offs[i + 1]], ref[i]), (streams, mode, v)
        finally:
            ctx.close()
