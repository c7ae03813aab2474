"""shard.ListExchange over gloo (world_size 2 and 3, CPU): the learned block
capacity, the regrow-and-gather-again path, and 32-bit narrowing at n = 32
(sets holding variable 31, the bit that sign-extends through int32).  Lists
are built directly (synthetic sets and scores per variable), so each case
checks the exchange alone: every rank must reassemble exactly the
single-rank lists in variable order."""
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


def _lists(n, seed, sizes):
    """Per variable v: sizes[v] distinct parent sets of the other variables
    (every third one holds the top variable n-1) with float32 scores."""
    rng = np.random.default_rng(seed)
    out = []
    for v in range(n):
        others = [b for b in range(n) if b != v]
        seen, sets = set(), []
        while len(sets) < sizes[v]:
            k = int(rng.integers(0, 4))
            bits = rng.choice(others, size=k, replace=False) if k else []
            s = 0
            for b in bits:
                s |= 1 << int(b)
            if len(sets) % 3 == 2 and v != n - 1:
                s |= 1 << (n - 1)
            if s not in seen:
                seen.add(s)
                sets.append(s)
        sc = rng.standard_normal(len(sets)).astype(np.float32) * -1000.0
        out.append((np.array(sets, dtype=np.uint64), sc))
    return out


def _single(n, lists):
    offs = np.zeros(n + 1, dtype=np.int64)
    for v in range(n):
        offs[v + 1] = offs[v] + len(lists[v][0])
    return offs, np.concatenate([l[0] for l in lists]), np.concatenate([l[1] for l in lists])


def _worker(rank, world, port, out_dir, n, steps):
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = [(1 << n) - 1] * n
    parts = shard.assign(n, world, full, 3)
    ex = shard.ListExchange(n, parts, full, 3, rank, device="cpu")
    rec = []
    for i, (seed, sizes) in enumerate(steps):
        lists = _lists(n, seed, sizes)
        offs = [0]
        for v in ex.mine:
            offs.append(offs[-1] + len(lists[v][0]))
        ex.fill_host(offs, np.concatenate([lists[v][0] for v in ex.mine]),
                     np.concatenate([lists[v][1] for v in ex.mine]))
        ex.allgather()
        o, st, sc = ex.assemble()
        np.savez(os.path.join(out_dir, f"r{rank}_s{i}.npz"), o=o, s=st.numpy().view(np.uint64), c=sc.numpy(),
                 block=ex.block, cap=ex.cap, regathers=ex.regathers)
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, world, n, steps):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), n, steps), nprocs=world, join=True,
                       start_method="spawn")
    res = []
    for i, (seed, sizes) in enumerate(steps):
        offs, sets, scores = _single(n, _lists(n, seed, sizes))
        for r in range(world):
            d = np.load(tmp_path / f"r{r}_s{i}.npz")
            assert np.array_equal(d["o"], offs), (i, r)
            assert np.array_equal(d["s"], sets), (i, r)
            assert d["c"].tobytes() == scores.tobytes(), (i, r)
        res.append(np.load(tmp_path / f"r0_s{i}.npz"))
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_learned_capacity_shrinks_blocks(tmp_path, world):
    """The first gather uses the a-priori bound (every scored set stored);
    the next ones use the largest gathered count plus slack."""
    n = 12
    steps = [(9800, [20] * n), (9800, [20] * n), (9801, [18] * n)]
    r = _run(tmp_path, world, n, steps)
    need = 20 * ((n + world - 1) // world)  # the largest rank's stored count
    assert int(r[0]["cap"]) > need + int(0.02 * need) + 256  # the a-priori bound
    assert int(r[1]["cap"]) == need + int(0.02 * need) + 256 and int(r[1]["block"]) < int(r[0]["block"])
    assert int(r[2]["regathers"]) == 0


@pytest.mark.parametrize("world", [2, 3])
def test_outgrown_capacity_regathers(tmp_path, world):
    """Lists that outgrow the learned capacity: every rank sees the counts in
    the gathered headers, grows the blocks and gathers once more."""
    n = 12
    steps = [(9810, [3] * n), (9811, [3] * n), (9812, [90] * n), (9813, [90] * n)]
    r = _run(tmp_path, world, n, steps)
    assert int(r[2]["regathers"]) == 1 and int(r[3]["regathers"]) == 1


def test_n32_sets_with_bit_31_survive_narrowing(tmp_path):
    """n = 32: sets travel as their low 32 bits; variable 31 is the sign bit
    of the int32 view and must come back as an unsigned mask."""
    n = 32
    steps = [(9820, [9] * n), (9821, [9] * n)]
    _run(tmp_path, 2, n, steps)
    _, sets, _ = _single(n, _lists(n, 9820, [9] * n))
    assert any(int(s) >> 31 for s in sets)
