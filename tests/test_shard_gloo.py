"""Multi-rank path on the CPU (gloo, world_size 2 and 3): variables striped
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


def _worker(rank, world, port, result_dir):
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import oracle
    import shard
    import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 9
    X, _ = synth.gaussian_sem(n, 1200, 9500)
    ds = oracle.Dataset(X)
    mine = shard.stripe(n, world, rank)
    offs = [0]
    sets, scores = [], []
    for v in mine:
        s, sc = ds.score_variable(2.0, v, (1 << n) - 1, 3)
        sets.append(s)
        scores.append(sc)
        offs.append(offs[-1] + len(s))
    packed = shard.pack(mine, offs, np.concatenate(sets), np.concatenate(scores))
    gathered = shard.allgather_lists(packed, world)
    o, st, sc = shard.unpack(gathered, n)
    np.savez(os.path.join(result_dir, f"r{rank}.npz"), o=o, s=st, c=sc)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_lists_equal_single_rank(tmp_path, oracle_built, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    import synth
    n = 9
    X, _ = synth.gaussian_sem(n, 1200, 9500)
    offs, sets, scores = oracle_built.Dataset(X).score_all(2.0, [(1 << n) - 1] * n, 3)
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
