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


def _sharded_worker(rank, world, port, result_dir, seed, n, extra):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "urlearning-cpp_amd"))
    import torch.distributed as dist
    import shard
    import synth as sy
    import ulg as u
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, W = sy.gaussian_sem(n, 3000, seed)
    rows = [r & ~(1 << i) for i, r in enumerate(sy.true_skeleton_edges(W, extra, seed))]
    ctx = u.Context(0)
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), u.candidates_from_edges(rows, n), 4)
    ctx.search_from_scores()
    res = shard.triplet_sharded(ctx, rows, world, rank)
    np.savez(os.path.join(result_dir, f"t{rank}.npz"), mec=res["mec"],
             st=np.array([res["runs"], res["distinct"], res["solved_here"], res["clusters"]]))
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("seed,n,extra", [(9410, 16, 0.1), (9411, 20, 0.15)])
def test_triplet_sharded_over_two_ranks_equals_one_gpu(ulg_ctx, tmp_path, seed, n, extra):
    """the first sweep's clusters solved once each over 2 ranks
    (one libulg context per rank, gloo exchange), then the driver on every
    rank: the MEC equals the single-GPU driver's, and the driver searches
    only what the exchange did not cover."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    mp.start_processes(_sharded_worker, args=(world, port, str(tmp_path), seed, n, extra), nprocs=world,
                       join=True, start_method="spawn")
    X, W = synth.gaussian_sem(n, 3000, seed)
    rows = [r & ~(1 << i) for i, r in enumerate(synth.true_skeleton_edges(W, extra, seed))]
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), ulg.candidates_from_edges(rows, n), 4)
    ulg_ctx.search_from_scores()
    one = ulg_ctx.triplet(edges=rows)
    clusters = ulg_ctx.triplet_clusters(rows)
    assert len(clusters) > world
    solved = 0
    for r in range(world):
        d = np.load(tmp_path / f"t{r}.npz")
        assert d["mec"].tolist() == one["mec"].tolist()
        runs, distinct, here, ncl = (int(x) for x in d["st"])
        assert runs == one["runs"] and ncl == len(clusters)
        assert distinct <= one["distinct"]
        solved += here
    assert solved == len(clusters)


def test_triplet_memo_reuse_and_put(ulg_ctx):
    """A memo seeded by ulg_triplet_memo_put (here: from a second context)
    leaves the driver nothing to search for those clusters, same MEC."""
    n = 14
    X, W = synth.gaussian_sem(n, 3000, 9412)
    rows = [r & ~(1 << i) for i, r in enumerate(synth.true_skeleton_edges(W, 0.1, 9412))]
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), ulg.candidates_from_edges(rows, n), 4)
    ulg_ctx.search_from_scores()
    one = ulg_ctx.triplet(edges=rows)
    again = ulg_ctx.triplet(edges=rows)  # same lists: the context's memo answers every run
    assert again["mec"].tolist() == one["mec"].tolist() and again["distinct"] == 0 and again["expanded"] == 0
    clusters = ulg_ctx.triplet_clusters(rows)
    par, st = ulg_ctx.triplet_solve(clusters)
    # the driver asked for some of them (orientations grow clusters mid-sweep,
    # so not necessarily all): only the rest are searched, and only once
    assert st["distinct"] < len(clusters)
    par2, st2 = ulg_ctx.triplet_solve(clusters)
    assert st2["distinct"] == 0 and np.array_equal(par2, par)
    other = ulg.Context(0)
    try:
        other.load(X, 2.0)
        other.score(list(range(n)), ulg.candidates_from_edges(rows, n), 4)
        other.search_from_scores()
        p2, st2 = other.triplet_solve(clusters)
        assert np.array_equal(p2, par) and st2["distinct"] == len(set(int(c) for c in clusters))
        other.search_from_scores()  # new lists: memo cleared
        other.triplet_memo_put(clusters, par)
        res = other.triplet(edges=rows)
        assert res["mec"].tolist() == one["mec"].tolist()
        assert res["distinct"] == one["distinct"] - (len(clusters) - st["distinct"])
    finally:
        other.close()


def test_triplet_look_ahead_threads_equal_sequential(ulg_ctx, oracle_built, monkeypatch):
    """The first sweep's look-ahead searches on host threads (host-built
    pattern databases, results held until the driver asks) give the
    sequential driver's MEC and statistics, and both equal the oracle's."""
    o = oracle_built
    n = 18
    X, W = synth.gaussian_sem(n, 3000, 9413)
    rows = [r & ~(1 << i) for i, r in enumerate(synth.true_skeleton_edges(W, 0.15, 9413))]
    offs, sets, costs = _oracle_costs(o, X, 2.0, 3, ulg.candidates_from_edges(rows, n))
    res = {}
    for threads in ("1", "8"):
        monkeypatch.setenv("ULG_TRIPLET_THREADS", threads)
        ulg_ctx.search_load(offs, sets, costs)
        res[threads] = ulg_ctx.triplet(edges=rows)
    ref = o.triplet(o.Search(n, offs, sets, costs), edges=rows)
    for r in res.values():
        assert r["mec"].tolist() == ref["mec"].tolist()
        assert (r["runs"], r["distinct"], r["expanded"]) == (ref["runs"], ref["distinct"], ref["expanded"])


def test_triplet_running_time_budget(ulg_ctx):
    """triplet_astar -r (triplet_astar.cpp:1674-1681): once the watchdog has
    fired every A* of the driver ends without a goal (:139-142,355,657-662),
    so process_triple sees the empty optimal-parents vectors of :855 and
    orients nothing -- memoised clusters included, which the reference would
    search again.  Full skeleton, n=16: every triple asks for the one
    16-variable cluster, whose search (2^16 lattice nodes) outlasts a 1 ms
    budget, so no run finds a goal and the MEC is empty; a generous budget
    changes nothing."""
    n = 16
    X, _ = synth.gaussian_sem(n, 3000, 9413)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), full, 3)
    ulg_ctx.search_from_scores()
    ref = ulg_ctx.triplet(edges=full)
    assert ulg_ctx.info("out_of_time") == 0 and ref["distinct"] == 1 and ref["mec"].any()
    try:
        ulg_ctx.set_option("time_limit_ms", 600000)
        same = ulg_ctx.triplet(edges=full)
        assert ulg_ctx.info("out_of_time") == 0 and same["mec"].tolist() == ref["mec"].tolist()
        ulg_ctx.search_from_scores()  # new lists: the memo starts empty again
        ulg_ctx.set_option("time_limit_ms", 1)
        cut = ulg_ctx.triplet(edges=full)
        assert ulg_ctx.info("out_of_time") == 1
        assert cut["distinct"] == 0 and cut["runs"] == ref["runs"]
        assert not cut["mec"].any()
    finally:
        ulg_ctx.set_option("time_limit_ms", 0)


def test_triplet_budget_interrupts_a_running_search(ulg_ctx):
    """-r bounds the wall clock: the reference's A* loop stops inside the
    search once outOfTime is set (triplet_astar.cpp:355), so a budget shorter
    than one cluster's search ends the call early instead of after that
    search.  Full skeleton: one n-variable cluster (2^n lattice nodes),
    n = 22, or 24 when the host searches n = 22 in under 0.2 s (so the cut is
    always measured); with a budget of a tenth of the uncut call's time the
    call returns well before the uncut search would finish, with the empty
    MEC."""
    import time
    for n in (22, 24):
        X, _ = synth.gaussian_sem(n, 2000, 9417)
        full = [(1 << n) - 1] * n
        ulg_ctx.load(X, 2.0)
        ulg_ctx.score(list(range(n)), full, 3)
        ulg_ctx.search_from_scores()
        t0 = time.perf_counter()
        ref = ulg_ctx.triplet(edges=full)
        uncut = time.perf_counter() - t0
        assert ulg_ctx.info("out_of_time") == 0 and ref["distinct"] == 1
        if uncut >= 0.2:
            break
    # the host's speed sets the uncut time (n = 22: 0.55-1.5 s across boxes)
    assert uncut >= 0.2, f"uncut n={n} search took {uncut:.3f} s: too short to measure a cut"
    try:
        budget_ms = max(20, int(100 * uncut))
        ulg_ctx.search_from_scores()  # an empty memo: the cluster is searched again
        ulg_ctx.set_option("time_limit_ms", budget_ms)
        t0 = time.perf_counter()
        cut = ulg_ctx.triplet(edges=full)
        dt = time.perf_counter() - t0
        assert ulg_ctx.info("out_of_time") == 1
        assert cut["distinct"] == 0 and not cut["mec"].any()
        assert dt < 0.5 * uncut, (dt, uncut, budget_ms)
    finally:
        ulg_ctx.set_option("time_limit_ms", 0)


def test_pdb_host_cancel_flag(ulg_ctx):
    """The look-ahead pool's host pattern database (pdb_host) stops on the
    pool's cancel flag and says so: built normally it equals the
    device PDB entry for entry; with the flag set before the build it reports
    cancelled and builds nothing (the pool then ends that search as
    cancelled, triplet_host.cpp SearchPool::work)."""
    n = 14
    X, _ = synth.gaussian_sem(n, 3000, 9418)
    full = [(1 << n) - 1] * n
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), full, 4)
    ulg_ctx.search_from_scores()
    cluster = (1 << n) - 1
    built, cancelled, entries, same = ulg_ctx.diag_pdb_host(cluster, 2, False)
    assert built == 1 and cancelled == 0 and entries == 2 ** 7 + 2 ** 7 and same == entries
    built, cancelled, entries, same = ulg_ctx.diag_pdb_host(cluster, 2, True)
    assert cancelled == 1 and entries == 0
    # a smaller cluster: the flag works whatever the group sizes
    built, cancelled, entries, same = ulg_ctx.diag_pdb_host(0b1011011101, 2, False)
    assert built == 1 and cancelled == 0 and same == entries > 0
