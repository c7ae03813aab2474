"""The configuration bench.py times, against the oracle command lines' C3
lists (tests/golden/c3_oracle.json).

* 3 contexts with one stream each, calls queued with ulg_cbic_score_async and
  collected two calls later, graph replays included: every context is left
  with the oracle's C3 lists.
* A captured call replayed as a hipGraph stores the same lists and scores bit
  for bit as the first (eager) call.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c3_oracle.json")


def _c3_digest_check(offs, sets, ref):
    for v in range(25):
        s = np.sort(np.asarray(sets[offs[v]:offs[v + 1]]).astype(np.uint64))
        assert len(s) == ref["stored_per_variable"][v], v
        assert hashlib.sha256(s.tobytes()).hexdigest() == ref["sets_sha256_per_variable"][v], v


@pytest.mark.timeout(300)
def test_c3_graph_replay_equals_first_call(ulg_ctx):
    ref = json.load(open(FIXTURE))
    n = 25
    X, _ = synth.gaussian_sem(n, 10000, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    first = ulg_ctx.score_all(list(range(n)), full, 6)
    again = ulg_ctx.score_all(list(range(n)), full, 6)
    for a, b in zip(first, again):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    _c3_digest_check(first[0], first[1], ref)


@pytest.mark.timeout(300)
def test_bench_configuration_slots_match_oracle():
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
