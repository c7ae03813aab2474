"""BASELINE configs C4 and C5 on the HIP path, against the CPU oracle.

C4: n=30, N=100k, MMPC skeleton (ulg_mmpc, alpha 0.01; equal to the
    oracle's ora_mmpc), 2-hop candidate sets (score_main.cpp:146-153), the
    reference's default parent limit -p = n - 1 (score_main.cpp:296-298):
    up to 18 candidates, so layers 9..18 run the wide kernels.
C5: n=32, N=50k, full skeleton.  As specified it is degenerate:
    -p defaults to 31 (2^31 sets per variable), and every triplet cluster
    has 32 > 26 variables, so triplet_astar skips every triple
    (triplet_astar.cpp:837-844) and the MEC is empty.  The scorer runs the
    k = 6 variant: 30,164,768 parent sets.

tests/golden/c45_oracle.json (make_c45_fixture.py) holds, for every C4
variable (30) and 8 C5 variables, the oracle's stored-set count, a SHA-256 of the
sorted masks, the score sum and every 512th (set, score).  The GPU must store
exactly those sets, with every sampled score within 1e-6 relative.  On every
variable of C5 the lists must also have the shape the reference produces
(order, the empty set, no self-parent, finite scores), and sampled sets
of every layer and both N4 phases are re-decided one by one by the oracle
(ora_decide against the cache the GPU left).  The C5 .pss text the GPU
formats equals the oracle's .pss writer on the same lists, byte for byte."""
import hashlib
import json
import math
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c45_oracle.json")


def _fixture():
    if not os.path.exists(FIXTURE):
        pytest.fail("tests/golden/c45_oracle.json missing: run tests/golden/make_c45_fixture.py")
    return json.load(open(FIXTURE))


def _check_against_fixture(fx, offs, sets, scores, vars_order, stride):
    where = {v: i for i, v in enumerate(vars_order)}
    for vs, ref in fx["per_variable"].items():
        i = where[int(vs)]
        s = sets[offs[i]:offs[i + 1]].astype(np.uint64)
        f = scores[offs[i]:offs[i + 1]]
        order = np.argsort(s, kind="stable")
        s, f = s[order], f[order]
        assert len(s) == ref["stored"], vs
        assert hashlib.sha256(s.tobytes()).hexdigest() == ref["sets_sha256"], vs
        tot = float(np.sum(f.astype(np.float64)))
        assert abs(tot - ref["score_sum"]) <= 1e-6 * max(abs(ref["score_sum"]), 1.0), vs
        assert [int(x) for x in s[::stride]] == ref["sample_sets"], vs
        for got, want in zip(f[::stride], ref["sample_scores"]):
            assert abs(float(got) - want) <= 1e-6 * max(abs(want), 1e-30), (vs, float(got), want)


@pytest.mark.timeout(600)
def test_c4_default_parent_limit_matches_oracle(ulg_ctx):
    top = _fixture()
    fx = top["c4"]
    n, N, k = fx["n"], fx["N"], fx["k"]
    X, _ = synth.gaussian_sem(n, N, 9200)
    ulg_ctx.load(X, 2.0)
    rows = ulg_ctx.mmpc(fx["alpha"])
    assert rows == fx["skeleton_rows"]  # the GPU MMPC equals the oracle's
    import ulg
    cands = ulg.candidates_from_edges(rows, n)
    assert max(bin(c & ~(1 << v)).count("1") for v, c in enumerate(cands)) > 8  # wide layers run
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), cands, k)
    _check_against_fixture(fx, offs, sets, scores, list(range(n)), top["sample_stride"])
    for vs, ref in fx["per_variable"].items():
        assert cands[int(vs)] == ref["candidates"], vs


@pytest.mark.timeout(900)
def test_c5_k6_matches_oracle_and_is_well_formed(ulg_ctx, oracle_built, tmp_path):
    top = _fixture()
    fx = top["c5"]
    n, N, k = fx["n"], fx["N"], fx["k"]
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    stored, scored = ulg_ctx.score(list(range(n)), full, k)
    assert scored == n * sum(math.comb(n - 1, L) for L in range(k + 1)) == 30164768  # SURVEY 8a, empty sets included
    offs, sets, scores = ulg_ctx.fetch(stored)
    _check_against_fixture(fx, offs, sets, scores, list(range(n)), top["sample_stride"])
    # shape of every variable's list (score_calculator.cpp:54-135, BIC_OLS.cpp:213-249)
    for v in range(n):
        s = sets[offs[v]:offs[v + 1]].astype(np.uint64)
        f = scores[offs[v]:offs[v + 1]]
        assert len(s) >= 1 and int(s[0]) == 0 and f[0] == 0.0, v  # the empty set, first
        pc = np.bitwise_count(s)
        assert np.all(np.diff(pc) >= 0) and pc.max() <= k, v
        for L in range(1, k + 1):  # Gosper order = increasing value inside a layer
            assert np.all(np.diff(s[pc == L].astype(np.uint64)) > 0), (v, L)
        assert not np.any((s >> np.uint64(v)) & np.uint64(1)), v
        # stored values are -ts: negative for sets worse than the empty set
        # (score_calculator.cpp:111), positive for accepted sets (BIC_OLS.cpp:249)
        assert np.all(np.isfinite(f)), v
    # the oracle re-decides sampled sets of every layer and both N4 phases
    ds = oracle_built.Dataset(X)
    rng = np.random.default_rng(32)
    checked = stored_hits = 0
    for v in (0, 9, 31):
        s_v, f_v = sets[offs[v]:offs[v + 1]], scores[offs[v]:offs[v + 1]]
        cache = oracle_built.Cache(s_v, f_v)
        gpu = {int(a): np.float32(b) for a, b in zip(s_v, f_v)}
        others = [u for u in range(n) if u != v]
        picks = []
        for L in range(1, k + 1):
            for with0 in ((True, False) if v != 0 else (False,)):
                pool = [u for u in others if u != 0]
                for _ in range(20):
                    P = sum(1 << int(u) for u in rng.choice(pool, size=L - 1 if with0 else L, replace=False))
                    picks.append(P | (1 if with0 else 0))
        picks += [int(x) for x in rng.choice(s_v, size=min(100, len(s_v)), replace=False)]
        for P in picks:
            st, val = ds.decide(2.0, v, P, cache)
            assert st == (P in gpu), (v, P, val)
            if st:
                g = float(gpu[P])
                assert abs(g - val) <= 1e-6 * max(abs(val), 1e-30), (v, P, g, val)
                stored_hits += 1
            checked += 1
    assert checked >= 800 and stored_hits >= 250
    # the .pss text the GPU formats (11 M lines) equals the oracle's writer
    # (score_main.cpp:173-203,383-400) on the same lists, byte for byte
    names = [str(i) for i in range(n)]
    ref = tmp_path / "c5_ref.pss"
    oracle_built.write_pss(str(ref), names, [N] * n, offs, sets, scores, num_records=N, parent_limit=k)
    ref_text = ref.read_bytes()
    ref.unlink()
    header = ref_text[: ref_text.index(b"VAR ")].decode()
    got = ulg_ctx.pss_format(header, names, [N] * n)
    assert len(got) == len(ref_text)
    assert hashlib.sha256(got).hexdigest() == hashlib.sha256(ref_text).hexdigest()


@pytest.mark.timeout(600)
def test_c5_full_skeleton_triplet_mec_is_empty(ulg_ctx):
    """with the full 32-variable skeleton every triple's cluster
    exceeds 26 variables (triplet_astar.cpp:837-844), so no A* runs and the
    MEC has no edge."""
    n, N, k = 32, 50000, 6
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), full, k)
    ulg_ctx.search_from_scores()
    res = ulg_ctx.triplet(edges=full)
    assert res["runs"] == 0 and res["distinct"] == 0 and res["expanded"] == 0
    assert not res["mec"].any()
