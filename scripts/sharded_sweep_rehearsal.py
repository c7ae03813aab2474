#!/usr/bin/env python3
"""The table-sharded GPU sweep (SURVEY 8e's n >= 31 path, ulg_sweep_shard_*)
rehearsed near C5's size on ONE GPU: `world` ranks (gloo, all on cuda:0) each
build the best-score tables and sweep slices of their own variables only and
combine every layer's (cost, leaf) keys with one MIN all-reduce; then, after
the ranks have exited and freed their tables, this process runs the
single-GPU sweep over all tables.  Prints one JSON line: per-rank times, the
per-layer all-reduce bytes, and whether cost bits, order, parent sets and the
reached-node count are identical.

    python scripts/sharded_sweep_rehearsal.py [n] [world] [k]   (default 30 2 2)
"""
import json
import os
import socket
import sys
import tempfile
import time
from math import comb

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
N, SEED = 5000, 9762


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out_dir, n, k):
    sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import shard
    import synth
    import ulg
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, _ = synth.gaussian_sem(n, N, SEED)
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
    own = shard.table_owners(n, world)[rank]
    # a budget for this rank's own tables only (12 B per entry, table_budget_kb):
    # the all-variable build on load is refused (the lists stay loaded)
    ctx.set_option("table_budget_kb", ((bin(own).count("1") << (n - 1)) * 12 >> 10) + 1024)
    ctx.search_from_scores()
    dist.barrier()
    t0 = time.perf_counter()
    res = shard.sharded_sweep(ctx, n, own, device="cuda", comm_device="cpu")
    dt = time.perf_counter() - t0
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), cost=np.float32(res["cost"]), vpar=res["vpar"],
             order=res["order"], exp=np.int64(res["expanded"]), own=np.uint64(own), sec=dt)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    import synth
    import ulg
    with tempfile.TemporaryDirectory() as td:
        t0 = time.perf_counter()
        mp.start_processes(worker, args=(world, _port(), td, n, k), nprocs=world, join=True, start_method="spawn")
        t_ranks = time.perf_counter() - t0
        parts = [dict(np.load(os.path.join(td, f"s{r}.npz"))) for r in range(world)]
    X, _ = synth.gaussian_sem(n, N, SEED)
    ctx = ulg.Context(0)
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), [(1 << n) - 1] * n, k)
    ctx.set_option("table_budget_kb", ((n << (n - 1)) * 12 >> 10) + 1024)  # every table on this GPU
    ctx.search_from_scores()
    t0 = time.perf_counter()
    ref = ctx.astar(edges=[(1 << n) - 1] * n, mode=1, net_text=False)
    t_single = time.perf_counter() - t0
    ctx.close()
    same = all(np.float32(p["cost"]).tobytes() == np.float32(ref["cost"]).tobytes()
               and [int(x) for x in p["order"]] == [int(x) for x in ref["order"]]
               and [int(x) for x in p["vpar"]] == [int(x) for x in ref["vpar"]]
               and int(p["exp"]) == ref["expanded"] for p in parts)
    owned = 0
    for p in parts:
        owned |= int(p["own"])
    print(json.dumps({
        "config": f"n={n}, N={N}, k={k}, lambda 2, full skeleton, seed {SEED}; {world} ranks (gloo) on one GPU",
        "identical_to_single_gpu": bool(same), "owned_partition": owned == (1 << n) - 1,
        "rank_sweep_s": [float(p["sec"]) for p in parts], "ranks_wall_s": t_ranks,
        "single_gpu_sweep_s": t_single, "goal_cost": float(ref["cost"]), "lattice_nodes": 1 << n,
        "allreduce_bytes_per_rank": 8 * sum(comb(n, L) for L in range(1, n + 1)),
        "largest_layer_keys": comb(n, n // 2),
        "tables_per_rank_bytes": [8 * bin(int(p["own"])).count("1") << (n - 1) for p in parts],
        "note": "rank_sweep_s includes the rank's own tables + sweep slices build and n gloo all-reduces "
                "through host memory (RCCL over xGMI on separate GPUs)"}), flush=True)


if __name__ == "__main__":
    main()
