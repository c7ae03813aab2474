"""GPU parity of the wide scorer layers (parent sets larger than
ULG_UNROLLED_PARENTS_GPU = 8, up to ULG_MAX_PARENTS_GPU = 31).

The reference's default parent limit is n - 1 (score_main.cpp:296-298), so
config C1 (data/hepatitis.clean.csv, n = 20) scores layers 1..19.  Layers
above 8 run the runtime-L kernels of cbic.hip (score_wide_kernel +
walk_wide_kernel, the explicit-stack replay of find_best_subset_score,
BIC_OLS.cpp:125-172).

Bar as in test_gpu_cbic.py: stored sets bit-exact, scores within 1e-6
relative.  Small configurations compare against the oracle run here; C1
compares against tests/golden/c1_hepatitis_digest.json, the oracle's full run
reduced to per-variable digests by tests/golden/make_c1_digest.py (the oracle
needs tens of CPU-minutes for it)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_gpu_cbic import _compare_lists, _oracle_lists, REL_TOL
import synth

pytestmark = pytest.mark.gpu


def load_csv_ascii(path):
    """Armadillo csv_ascii as the reference loads it: rows = lines,
    a non-numeric token (the header) reads as 0.  Same rule as host/io.cpp."""
    with open(path) as f:
        lines = [ln.rstrip("\r\n") for ln in f]
    n = max(ln.count(",") + 1 for ln in lines)
    X = np.zeros((len(lines), n), dtype=np.float64)
    for r, ln in enumerate(lines):
        for c, tok in enumerate(ln.split(",")):
            try:
                X[r, c] = float(tok)
            except ValueError:
                pass
    return X


@pytest.mark.parametrize("seed,n,N,k", [(9210, 11, 2000, 10), (9211, 12, 1500, 11), (9212, 13, 3000, 9),
                                        (9213, 14, 1000, 13)])
def test_wide_layers_full_skeleton_match_oracle(ulg_ctx, oracle_built, seed, n, N, k):
    X, _ = synth.gaussian_sem(n, N, seed)
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    g = ulg_ctx.score_all(variables, cands, k)
    o = _oracle_lists(oracle_built, X, 2.0, variables, cands, k)
    _compare_lists(*o, *g, variables, ctx=f"seed {seed} k={k}")


@pytest.mark.parametrize("lam", [0.5, 2.0])
def test_wide_layers_hepatitis_prefix_match_oracle(ulg_ctx, oracle_built, lam):
    """The C1 data on its first 13 columns at k = 12: weak-signal data where
    many large sets survive (the walk-heavy case)."""
    X = load_csv_ascii(os.path.join(GOLDEN, "hepatitis.clean.csv"))[:, :13]
    n = X.shape[1]
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, lam)
    g = ulg_ctx.score_all(variables, cands, n - 1)
    o = _oracle_lists(oracle_built, X, lam, variables, cands, n - 1)
    _compare_lists(*o, *g, variables, ctx=f"hepatitis[:, :13] lam={lam}")


@pytest.mark.parametrize("lam", [0.5, 2.0])
def test_wide_lds_replay_every_walk_hepatitis_prefix_match_oracle(ulg_ctx, oracle_built, lam):
    """wide_lds = 2 sends every wide walk to walk_wide_lds_kernel (the mask-frame
    replay with skip / hi bitsets), not only the long ones: its lists must
    equal the oracle's on the walk-heavy hepatitis prefix."""
    X = load_csv_ascii(os.path.join(GOLDEN, "hepatitis.clean.csv"))[:, :13]
    n = X.shape[1]
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    ulg_ctx.load(X, lam)
    try:
        ulg_ctx.set_option("wide_lds", 2)
        g = ulg_ctx.score_all(variables, cands, n - 1)
    finally:
        ulg_ctx.set_option("wide_lds", 1)
    o = _oracle_lists(oracle_built, X, lam, variables, cands, n - 1)
    _compare_lists(*o, *g, variables, ctx=f"hepatitis[:, :13] lam={lam} wide_lds=2")


def test_c1_hepatitis_default_parent_limit_matches_digest(ulg_ctx):
    """Config C1 (BASELINE.json configs[0]) on the GPU: all 20 variables, full
    skeleton, -p default n - 1 = 19, against the oracle's digest."""
    with open(os.path.join(GOLDEN, "c1_hepatitis_digest.json")) as f:
        dig = json.load(f)
    X = load_csv_ascii(os.path.join(GOLDEN, dig["csv"]))
    n = X.shape[1]
    assert (X.shape[0], n) == (dig["N"], dig["n"])
    variables = list(range(n))
    cands = [(1 << n) - 1] * n
    for lam_s, per_var in dig["runs"].items():
        ulg_ctx.load(X, float(lam_s))
        offs, sets, scores = ulg_ctx.score_all(variables, cands, dig["max_parents"])
        for v in variables:
            d = per_var[v]
            s = sets[offs[v]:offs[v + 1]]
            sc = scores[offs[v]:offs[v + 1]]
            assert len(s) == d["count"], f"lam={lam_s} variable {v}: {len(s)} stored vs oracle {d['count']}"
            assert hashlib.sha256(np.ascontiguousarray(s, dtype=np.uint64).tobytes()).hexdigest() == d["sets_sha256"], \
                f"lam={lam_s} variable {v}: stored sets differ from the oracle's"
            tot = float(sc.astype(np.float64).sum())
            assert abs(tot - d["score_sum"]) <= REL_TOL * max(abs(d["score_sum"]), 1.0), (v, tot, d["score_sum"])
            for idx, (ps, pscore) in zip(np.unique(np.linspace(0, len(s) - 1, 64).astype(np.int64)), d["samples"]):
                assert int(s[idx]) == ps
                assert abs(float(sc[idx]) - pscore) <= REL_TOL * max(abs(pscore), 1.0), (v, ps, float(sc[idx]), pscore)


def test_wide_hicover_prune_identical_lists(ulg_ctx):
    """ulg_set_option("wide_prune"): the walks skip absent nodes below which no
    present key reaches -ts; "wide_reduced": they skip the recursion's no-op
    re-tests; "wide_lds": walks over 2^6 steps (2: over 1 step, so every
    walk) are replayed by walk_wide_lds_kernel.  The stored lists with and without either are identical bit for
    bit, on C4's (n=30, N=100k, MMPC, -p = n-1) variables
    whose unpruned walks finish in well under a second each."""
    import ulg
    n, N = 30, 100000
    X, _ = synth.gaussian_sem(n, N, 9200)
    ulg_ctx.load(X, 2.0)
    rows = ulg_ctx.mmpc(0.01)
    cands = ulg.candidates_from_edges(rows, n)
    vs = [10, 14, 29, 4, 16, 27]
    assert all(9 <= bin(cands[v] & ~(1 << v)).count("1") <= 12 for v in vs)
    out = []
    try:
        for prune, reduced, lds in ((0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (1, 1, 1), (1, 1, 2)):
            ulg_ctx.set_option("wide_prune", prune)
            ulg_ctx.set_option("wide_reduced", reduced)
            ulg_ctx.set_option("wide_lds", lds)
            offs, sets, scores = ulg_ctx.score_all(vs, [cands[v] for v in vs], n - 1)
            out.append((np.asarray(offs).copy(), np.asarray(sets).copy(), np.asarray(scores).copy()))
    finally:
        ulg_ctx.set_option("wide_prune", 1)
        ulg_ctx.set_option("wide_reduced", 1)
        ulg_ctx.set_option("wide_lds", 1)
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert np.array_equal(out[0][1], o[1])
        assert out[0][2].tobytes() == o[2].tobytes()


@pytest.mark.timeout(300)
def test_wide_pool_identical_lists_c4(ulg_ctx):
    """ulg_set_option("wide_pool"): the wide layers variable by variable on
    score_streams host threads, every stream group's part of a layer
    together, or picked by the candidate-count spread (2, default);
    "wide_host": LDS replays past that many iterations finish on host threads
    (1: every replay does, so host_walk re-decides all of them; 0: none) in
    launches of at most "wide_host_max" replays, "wide_host_first": launches
    of at most that many replays go to the host whole (and, with "wide_host_q",
    launches of <= 128 replays over 2^q >= 2^wide_host_q subsets), "wide_host_threads":
    host threads per launch.  All 30 C4 variables (n=30, N=100k, MMPC,
    -p = n-1; the wide layers reach 18) give bit-identical lists in every
    combination, and the pool's repeat call too."""
    import ulg
    n, N = 30, 100000
    X, _ = synth.gaussian_sem(n, N, 9200)
    ulg_ctx.load(X, 2.0)
    rows = ulg_ctx.mmpc(0.01)
    cands = ulg.candidates_from_edges(rows, n)
    vs = list(range(n))
    out = []
    defaults = dict(wide_pool=2, score_streams=3, wide_host=1024, wide_host_max=4096, wide_host_first=0,
                    wide_host_threads=16, wide_host_q=0)
    combos = [dict(wide_pool=0, wide_host=0), dict(), dict(), dict(wide_pool=1, wide_host=4096),
              dict(wide_pool=1, score_streams=2), dict(wide_pool=1, wide_host=1, wide_host_max=1 << 40),
              dict(wide_pool=0, score_streams=1, wide_host=64), dict(wide_host_first=64, wide_host_threads=3),
              dict(wide_host_q=14)]
    try:
        for combo in combos:
            for name, val in dict(defaults, **combo).items():
                ulg_ctx.set_option(name, val)
            offs, sets, scores = ulg_ctx.score_all(vs, [cands[v] for v in vs], n - 1)
            out.append((np.asarray(offs).copy(), np.asarray(sets).copy(), np.asarray(scores).copy()))
    finally:
        for name, val in defaults.items():
            ulg_ctx.set_option(name, val)
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert np.array_equal(out[0][1], o[1])
        assert out[0][2].tobytes() == o[2].tobytes()


@pytest.mark.timeout(400)
def test_c1_hepatitis_reference_defaults_lambda_half(ulg_ctx):
    """Config C1 at the reference's defaults: lambda 0.5 (score_main.cpp:214)
    and -p 19 on data/hepatitis.clean.csv.  The walks are far deeper than at
    lambda 2 (the GPU takes about 75 s; the oracle's literal recursion does
    not finish the 19 layers in hours), so tests/golden/c1_hepatitis_default.json
    holds the oracle run with -p K: every layer <= K of the GPU's -p 19 lists
    must equal it (a layer's stored sets depend only on the layers below)."""
    path = os.path.join(GOLDEN, "c1_hepatitis_default.json")
    if not os.path.exists(path):
        pytest.fail("tests/golden/c1_hepatitis_default.json missing: run tests/golden/make_c1_default_fixture.py")
    with open(path) as f:
        fx = json.load(f)
    X = load_csv_ascii(os.path.join(GOLDEN, fx["csv"]))
    n = X.shape[1]
    assert (X.shape[0], n) == (fx["N"], fx["n"])
    ulg_ctx.load(X, fx["lambda"])
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), [(1 << n) - 1] * n, fx["max_parents_run"])
    K = fx["layers_checked"]
    deeper = 0
    for v in range(n):
        d = fx["per_variable"][v]
        s = sets[offs[v]:offs[v + 1]]
        sc = scores[offs[v]:offs[v + 1]]
        pc = np.bitwise_count(s.astype(np.uint64))
        assert np.all(np.diff(pc) >= 0), v
        low = int(np.searchsorted(pc, K, side="right"))
        deeper += len(s) - low
        s, sc = s[:low], sc[:low]
        assert len(s) == d["count"], f"variable {v}: {len(s)} stored in layers <= {K} vs oracle {d['count']}"
        assert hashlib.sha256(np.ascontiguousarray(s, dtype=np.uint64).tobytes()).hexdigest() == d["sets_sha256"], v
        tot = float(sc.astype(np.float64).sum())
        assert abs(tot - d["score_sum"]) <= REL_TOL * max(abs(d["score_sum"]), 1.0), (v, tot, d["score_sum"])
        for idx, (ps, pscore) in zip(np.unique(np.linspace(0, len(s) - 1, 64).astype(np.int64)), d["samples"]):
            assert int(s[idx]) == ps
            assert abs(float(sc[idx]) - pscore) <= REL_TOL * max(abs(pscore), 1.0), (v, ps, float(sc[idx]), pscore)
    assert deeper > 0  # layers above K stored sets too (checked only through the GPU's own walk forms)
    # all 19 layers against the direct walk form (walk_wide_kernel, no LDS
    # replay), whose digest tests/golden/c1_hepatitis_default_walk_digest.json holds
    with open(os.path.join(GOLDEN, "c1_hepatitis_default_walk_digest.json")) as f:
        wd = json.load(f)
    assert wd["lambda"] == fx["lambda"] and wd["max_parents_run"] == fx["max_parents_run"]
    for v in range(n):
        d = wd["per_variable"][v]
        s = np.ascontiguousarray(sets[offs[v]:offs[v + 1]], dtype=np.uint64)
        sc = np.ascontiguousarray(scores[offs[v]:offs[v + 1]])
        assert len(s) == d["count"], v
        assert hashlib.sha256(s.tobytes()).hexdigest() == d["sets_sha256"], v
        assert hashlib.sha256(sc.tobytes()).hexdigest() == d["scores_sha256"], v
