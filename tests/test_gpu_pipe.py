"""The persistent scoring pipeline (score_pipe 1, csrc/cbic_pipe.hip: one
launch per call, per-variable stage chains released by device counters) and
the configuration the bench times.

* The pipeline stores exactly the oracle's parent sets (score_calculator.cpp:
  54-135 with BIC_OLS.cpp:125-276 restated in oracle/), on both N4 phases
  (candidate lists with and without variable 0), sparse candidate sets,
  every tile size, both compiled occupancies.
* At C3 it stores the oracle command lines' lists (tests/golden/c3_oracle.json)
  and the layer launches' lists bit for bit (scores included).
* The bench's timed configuration -- 3 contexts with one stream each, calls
  queued with ulg_cbic_score_async, graph replays included -- leaves every
  context with the oracle's C3 lists.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import synth
from test_gpu_cbic import _compare_lists, _oracle_lists

pytestmark = pytest.mark.gpu
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c3_oracle.json")


def _with_options(ctx, opts):
    """Set options, returning the previous values' restore list."""
    for k, v in opts.items():
        ctx.set_option(k, v)


def _c3_digest_check(offs, sets, ref):
    for v in range(25):
        s = np.sort(np.asarray(sets[offs[v]:offs[v + 1]]).astype(np.uint64))
        assert len(s) == ref["stored_per_variable"][v], v
        assert hashlib.sha256(s.tobytes()).hexdigest() == ref["sets_sha256_per_variable"][v], v


@pytest.mark.parametrize("opts", [
    dict(score_pipe=1),
    dict(score_pipe=1, pipe_rounds=1),
    dict(score_pipe=1, pipe_rounds_small=3),
    dict(score_pipe=1, pipe_occ=3),
    dict(score_pipe=1, score_small_layers=1),
    dict(score_pipe=1, score_small_layers=2, pipe_rounds=1),
])
def test_pipeline_matches_oracle(ulg_ctx, oracle_built, opts):
    cases = [(11, 2500, 6, "full"), (12, 3000, 6, "novar0"), (13, 3000, 5, "sparse"), (9, 2000, 3, "full")]
    try:
        _with_options(ulg_ctx, opts)
        for n, N, k, kind in cases:
            X, _ = synth.gaussian_sem(n, N, 9260 + n)
            ulg_ctx.load(X, 2.0)
            full = (1 << n) - 1
            if kind == "full":
                variables, cands = list(range(n)), [full] * n
            elif kind == "novar0":
                variables, cands = list(range(1, n)), [full & ~1] * (n - 1)
            else:
                rng = np.random.default_rng(n)
                variables = list(range(n))
                cands = [int(full & ~int(rng.integers(0, 1 << n))) | 1 for _ in range(n)]
            g = ulg_ctx.score_all(variables, cands, k)
            o = _oracle_lists(oracle_built, X, 2.0, variables, cands, k)
            _compare_lists(*o, *g, variables, ctx=f"{opts} n={n} {kind} k={k}")
    finally:
        for k in opts:
            ulg_ctx.set_option(k, {"score_pipe": 0, "pipe_rounds": 2, "pipe_rounds_small": 1, "pipe_occ": 2,
                                   "score_small_layers": 4}[k])


@pytest.mark.timeout(300)
def test_pipeline_c3_equals_oracle_and_layer_launches(ulg_ctx):
    ref = json.load(open(FIXTURE))
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    res = {}
    try:
        for pipe in (0, 1):
            ulg_ctx.set_option("score_pipe", pipe)
            res[pipe] = ulg_ctx.score_all(list(range(n)), full, 6)
        again = ulg_ctx.score_all(list(range(n)), full, 6)  # graph replay of the pipeline
    finally:
        ulg_ctx.set_option("score_pipe", 0)
    for a, b, c in zip(res[0], res[1], again):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes() == np.asarray(c).tobytes()
    _c3_digest_check(res[1][0], res[1][1], ref)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("pipe", [0, 1])
def test_bench_configuration_slots_match_oracle(pipe):
    """bench.py's timed loop: 3 contexts on one GPU, score_streams 1, each call
    queued with score_async and collected two calls later, 12 calls (so every
    context replays its captured graph); every context's lists equal the
    oracle fixture's."""
    import ulg
    ref = json.load(open(FIXTURE))
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    full = [(1 << n) - 1] * n
    ctxs = [ulg.Context(0) for _ in range(3)]
    try:
        for c in ctxs:
            c.set_option("score_streams", 1)
            c.set_option("score_pipe", pipe)
            c.load(X, 2.0)
        pend = []
        for i in range(12):
            c = ctxs[i % 3]
            c.score_async(list(range(n)), full, 6)
            pend.append(c)
            if len(pend) == 3:
                pend.pop(0).score_finish()
        for c in pend:
            c.score_finish()
        for c in ctxs:
            st, _ = c.score_finish()
            offs, sets, _ = c.fetch(st)
            _c3_digest_check(offs, sets, ref)
    finally:
        for c in ctxs:
            c.close()
