"""The multi-GPU scoring path on the HIP scorer, rehearsed on one
GPU: two ranks (gloo, both on cuda:0) each score their balanced share of the
variables through libulg, write the lists into their exchange block straight
from the scorer's device buffers (ulg_cbic_fetch, device pointers), run the
one all-gather and reassemble.  Every rank must end with exactly the lists a
single-rank ulg_cbic_score produces, and tables built from them
(ulg_search_load_scores) must give the single-rank search result."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

CASES = {
    # C2 at full size, and a C4-shaped sparse skeleton with very unequal
    # 2-hop candidate sets (balanced by parent-set counts, not v % ws)
    "c2": dict(n=20, N=10000, k=4, sparse=False),
    "sparse": dict(n=24, N=5000, k=8, sparse=True),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(case):
    import synth
    import ulg
    c = CASES[case]
    X, W = synth.gaussian_sem(c["n"], c["N"], 9700)
    if c["sparse"]:
        rows = synth.true_skeleton_edges(W, extra_frac=0.3, seed=3)
        cands = ulg.candidates_from_edges(rows, c["n"])
    else:
        rows, cands = None, [(1 << c["n"]) - 1] * c["n"]
    return c, X, rows, cands


def _worker(rank, world, port, out_dir, case):
    sys.path[:0] = [os.path.join(ROOT, "urlearning-cpp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import shard
    import ulg
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c, X, rows, cands = _setup(case)
    n, k = c["n"], c["k"]
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    parts = shard.assign(n, world, cands, k)
    ex = shard.ListExchange(n, parts, cands, k, rank, device="cuda", comm_device="cpu")
    stored, _ = ctx.score(ex.mine, [cands[v] for v in ex.mine], k)
    ex.fill(ctx, stored)
    ex.allgather()
    offs, sets, scores = ex.assemble(device="cuda")
    ctx.search_load_scores(offs, sets.data_ptr(), scores.data_ptr(), device_ptrs=True)
    res = ctx.astar(edges=rows if rows is not None else [(1 << n) - 1] * n, mode=1, net_text=False)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), o=offs, s=sets.cpu().numpy().view(np.uint64),
             c=scores.cpu().numpy(), cost=np.float32(res["cost"]), vpar=res["vpar"], mine=np.array(ex.mine))
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", sorted(CASES))
def test_hip_shard_exchange_equals_single_rank(tmp_path, ulg_ctx, case):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), case), nprocs=world, join=True,
                       start_method="spawn")
    c, X, rows, cands = _setup(case)
    n, k = c["n"], c["k"]
    ulg_ctx.load(X, 2.0)
    offs, sets, scores = ulg_ctx.score_all(list(range(n)), cands, k)
    ulg_ctx.search_from_scores()
    ref = ulg_ctx.astar(edges=rows if rows is not None else [(1 << n) - 1] * n, mode=1, net_text=False)
    mine = []
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(d["o"], offs), r
        assert np.array_equal(d["s"], sets), r
        assert d["c"].tobytes() == scores.tobytes(), r
        assert np.float32(d["cost"]).tobytes() == np.float32(ref["cost"]).tobytes(), r
        assert [int(x) for x in d["vpar"]] == [int(x) for x in ref["vpar"]], r
        mine.append(set(int(v) for v in d["mine"]))
    assert mine[0].isdisjoint(mine[1]) and mine[0] | mine[1] == set(range(n))


def _bench(args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_two_ranks_on_one_gpu_matches_one_rank():
    """bench.py --gpus 2 starts its own two ranks (gloo, both on GPU 0),
    reports n_gpus 2, and its gathered lists and goal cost equal N=1's."""
    common = ["--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench(["--gpus", "1"] + common)
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", "--device", "0"] + common)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["mode"] == "shard" and two["scaling"] == "strong"
    assert two["astar"]["ranks_agree"] is True
    assert two["astar"]["lists_sha256"] == one["astar"]["lists_sha256"]
    assert two["astar"]["gpu_search"]["goal_cost"] == one["astar"]["gpu_search"]["goal_cost"]
    assert two["shard_step"]["exchange_ms"] > 0
    assert two["astar"]["table_sharded_sweep"]["same_as_replica"] is True


def _sweep_worker(rank, world, port, out_dir, n, N, k, seed):
    sys.path[:0] = [os.path.join(ROOT, "urlearning-cpp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import shard
    import synth
    import ulg
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, _ = synth.gaussian_sem(n, N, seed)
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
    ctx.search_from_scores()
    masks = shard.table_owners(n, world)
    res = shard.sharded_sweep(ctx, n, masks[rank], device="cuda", comm_device="cpu")
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), cost=np.float32(res["cost"]), vpar=res["vpar"],
             order=res["order"], exp=np.int64(res["expanded"]), own=np.uint64(masks[rank]))
    # the tables are back to every variable for the next search on this context
    ctx.set_option("sweep_table", 1)
    again = ctx.astar(edges=[(1 << n) - 1] * n, mode=1, net_text=False)
    assert np.float32(again["cost"]).tobytes() == np.float32(res["cost"]).tobytes()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n,N,k,seed", [(2, 20, 10000, 4, 9200), (3, 22, 6000, 5, 9751),
                                              (2, 26, 5000, 3, 9760), (2, 28, 5000, 3, 9761)])
def test_table_sharded_sweep_equals_single_gpu(tmp_path, ulg_ctx, world, n, N, k, seed):
    """SURVEY 8e's n >= 31 path, rehearsed below n = 31: each rank holds the
    best-score tables and sweep slices of its own variables only
    (ulg_sweep_shard_begin), one MIN all-reduce per layer combines the ranks'
    (cost, leaf) keys.  Cost bits, order, parent sets and the reached-node
    count equal the single-GPU sweep's; the owned variables partition 0..n-1.
    n = 26 and 28 run the 32-bit colex and key paths near C5's sizes (the
    middle layer of n = 28 holds C(28, 14) = 40,116,600 nodes)."""
    import synth
    mp.start_processes(_sweep_worker, args=(world, _free_port(), str(tmp_path), n, N, k, seed), nprocs=world,
                       join=True, start_method="spawn")
    X, _ = synth.gaussian_sem(n, N, seed)
    ulg_ctx.load(X, 2.0)
    ulg_ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
    ulg_ctx.search_from_scores()
    ref = ulg_ctx.astar(edges=[(1 << n) - 1] * n, mode=1, net_text=False)
    owned = 0
    for r in range(world):
        d = np.load(tmp_path / f"s{r}.npz")
        assert np.float32(d["cost"]).tobytes() == np.float32(ref["cost"]).tobytes(), r
        assert [int(x) for x in d["order"]] == [int(x) for x in ref["order"]], r
        assert [int(x) for x in d["vpar"]] == [int(x) for x in ref["vpar"]], r
        assert int(d["exp"]) == ref["expanded"], r
        assert owned & int(d["own"]) == 0
        owned |= int(d["own"])
    assert owned == (1 << n) - 1
