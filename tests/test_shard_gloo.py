"""Multi-rank path on the CPU (gloo, world_size 2 and 3): variables balanced
over ranks, one all-gather of the per-variable lists, reassembly in
variable order -- identical to scoring every variable on one rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cands(n, sparse):
    import synth
    import ulg
    if not sparse:
        return [(1 << n) - 1] * n
    _, W = synth.gaussian_sem(n, 1200, 9500)
    return ulg.candidates_from_edges(synth.true_skeleton_edges(W), n)


def _worker(rank, world, port, result_dir, sparse):
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import oracle
    import shard
    import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, k = 9, 3
    X, _ = synth.gaussian_sem(n, 1200, 9500)
    cands = _cands(n, sparse)
    ds = oracle.Dataset(X)
    parts = shard.assign(n, world, cands, k)
    ex = shard.ListExchange(n, parts, cands, k, rank, device="cpu")
    offs = [0]
    sets, scores = [], []
    for v in ex.mine:
        s, sc = ds.score_variable(2.0, v, cands[v], k)
        sets.append(s)
        scores.append(sc)
        offs.append(offs[-1] + len(s))
    ex.fill_host(offs, np.concatenate(sets) if sets else np.zeros(0, np.uint64),
                 np.concatenate(scores) if scores else np.zeros(0, np.float32))
    ex.allgather()
    o, st, sc = ex.assemble()
    np.savez(os.path.join(result_dir, f"r{rank}.npz"), o=o, s=st.numpy().view(np.uint64), c=sc.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("sparse", [False, True])
def test_sharded_lists_equal_single_rank(tmp_path, oracle_built, world, sparse):
    """Balanced variable shards + the one all-gather of fixed-size blocks
    (shard.ListExchange): every rank ends with the single-rank lists."""
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), sparse), nprocs=world, join=True,
                       start_method="spawn")
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    import synth
    n = 9
    X, _ = synth.gaussian_sem(n, 1200, 9500)
    offs, sets, scores = oracle_built.Dataset(X).score_all(2.0, _cands(n, sparse), 3)
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(d["o"], offs)
        assert np.array_equal(d["s"], sets)
        assert d["c"].tobytes() == scores.tobytes()


def test_stripe_is_a_partition():
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    import shard
    for n in (1, 7, 25, 32):
        for ws in (1, 2, 4, 8):
            parts = [shard.stripe(n, ws, r) for r in range(ws)]
            assert sorted(v for p in parts for v in p) == list(range(n))


def test_assign_balances_parent_set_counts():
    """ranks balanced on sum_L C(m_v, L).  With the C4-shaped
    2-hop candidate sets of very different sizes, LPT keeps every rank within
    one variable's weight of the others, where v % ws does not."""
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    import shard
    n, k = 30, 29
    ms = [8, 8, 6, 13, 12, 2, 8, 16, 14, 18, 10, 8, 4, 14, 10, 13, 12, 9, 8, 6, 13, 13, 14, 17, 3, 14, 7, 12, 8, 10]
    cands = [sum(1 << ((v + 1 + j) % n) for j in range(m)) for v, m in enumerate(ms)]
    w = [shard.var_weight(n, v, cands[v], k) for v in range(n)]
    assert w == [2 ** m for m in ms]
    for ws in (1, 2, 4, 8):
        parts = shard.assign(n, ws, cands, k)
        assert parts == shard.assign(n, ws, cands, k)
        assert sorted(v for p in parts for v in p) == list(range(n))
        loads = [sum(w[v] for v in p) for p in parts]
        assert max(loads) - min(loads) <= max(w)
    # full skeleton: every variable weighs the same, so ranks differ by <= 1 variable
    full = [(1 << 25) - 1] * 25
    parts = shard.assign(25, 8, full, 6)
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_assign_clusters_is_a_balanced_deterministic_partition():
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    import shard
    rng = np.random.default_rng(9600)
    clusters = np.array([int(x) for x in rng.integers(1, 1 << 20, size=57)], dtype=np.uint64)
    for ws in (1, 2, 3, 8):
        own = shard.assign_clusters(clusters, ws)
        assert np.array_equal(own, shard.assign_clusters(clusters, ws))
        assert set(own.tolist()) <= set(range(ws))
        loads = [sum(1 << bin(int(c)).count("1") for c, o in zip(clusters, own) if o == r) for r in range(ws)]
        biggest = max(1 << bin(int(c)).count("1") for c in clusters)
        assert max(loads) - min(loads) <= biggest  # LPT: within one job of each other


def _memo_worker(rank, world, port, result_dir):
    """Each rank contributes the memo rows of the clusters it owns; after the
    one all-gather every rank holds every row (the exchange of
    shard.triplet_sharded, with a stand-in per-cluster result)."""
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    import torch.distributed as dist
    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 13
    rng = np.random.default_rng(9601)
    clusters = np.unique(rng.integers(1, 1 << n, size=40).astype(np.uint64))
    own = shard.assign_clusters(clusters, world)
    mine = clusters[own == rank]
    parents = np.array([[(int(c) * 2654435761 + v) & ((1 << n) - 1) for v in range(n)] for c in mine],
                       dtype=np.uint64).reshape(len(mine), n)
    cl, pa = shard.unpack_memo(shard.allgather_rows(shard.pack_memo(mine, parents, n), world))
    np.savez(os.path.join(result_dir, f"m{rank}.npz"), cl=cl, pa=pa, all=clusters)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_triplet_memo_exchange_complete_on_every_rank(tmp_path, world):
    mp.start_processes(_memo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    n = 13
    for r in range(world):
        d = np.load(tmp_path / f"m{r}.npz")
        order = np.argsort(d["cl"])
        assert np.array_equal(d["cl"][order], np.sort(d["all"]))
        for c, row in zip(d["cl"], d["pa"]):
            assert [int(x) for x in row] == [(int(c) * 2654435761 + v) & ((1 << n) - 1) for v in range(n)]


def test_table_owners_partition_balanced():
    import shard
    for n, ws in [(32, 8), (30, 4), (25, 3), (5, 8)]:
        masks = shard.table_owners(n, ws)
        assert len(masks) == ws
        acc = 0
        for m in masks:
            assert acc & m == 0
            acc |= m
        assert acc == (1 << n) - 1
        sizes = [bin(m).count("1") for m in masks]
        assert max(sizes) - min(sizes) <= 1  # full skeleton: every table is 2^(n-1)
    # a sparse skeleton: balanced on 2^{m_v}
    cands = [(1 << 10) - 1] + [0b11] * 9
    masks = shard.table_owners(10, 2, cands)
    assert masks[0] == 1 and masks[1] == ((1 << 10) - 1) & ~1
