"""Variable-sharded scoring across ranks (one process per GPU) and the single
exchange step of SURVEY 8e: every rank scores its stripe of the variables
(v % world_size == rank, as score_main.cpp:136-139 stripes threads), then one
all-gather (RCCL over xGMI on MI355X; gloo in the CPU tests) hands every rank
the complete per-variable (set, score) lists in variable order, ready for
ulg_search_load or a .pss writer.

Wire format per entry: int64 [variable, set, float32 score bits].

triplet_astar shards the same way: its distinct clusters are
independent exact A* problems (triplet_astar.cpp:285-674, one per cluster).
Every rank enumerates the first sweep's clusters (ulg_triplet_clusters),
solves its share (ulg_triplet_solve), one all-gather of [cluster, parents...]
rows fills every rank's memo (ulg_triplet_memo_put), and the sequential
driver (ulg_triplet_astar) then runs on each rank with nothing left to search
but the clusters that orientations add mid-sweep -- the MEC is the one a
single GPU computes."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def stripe(n: int, world_size: int, rank: int):
    return [v for v in range(n) if v % world_size == rank]


def pack(variables, offsets, sets, scores, device="cpu") -> torch.Tensor:
    """Local lists (variables[i] owns [offsets[i], offsets[i+1])) -> [count, 3] int64."""
    offsets = np.asarray(offsets, dtype=np.int64)
    count = int(offsets[-1])
    out = np.empty((count, 3), dtype=np.int64)
    for i, v in enumerate(variables):
        out[offsets[i]:offsets[i + 1], 0] = v
    out[:, 1] = np.asarray(sets[:count], dtype=np.uint64).view(np.int64)
    out[:, 2] = np.asarray(scores[:count], dtype=np.float32).view(np.int32).astype(np.int64)
    return torch.from_numpy(out).to(device)


def pack_device(variables, offsets: torch.Tensor, sets: torch.Tensor, scores: torch.Tensor) -> torch.Tensor:
    """Same as pack() for device tensors (ulg_cbic_fetch(device_ptrs=1) output):
    offsets int64 [nv+1], sets int64 (uint64 bits), scores float32."""
    count = int(offsets[-1].item())
    dev = sets.device
    per = (offsets[1:] - offsets[:-1]).to(torch.int64)
    var = torch.repeat_interleave(torch.as_tensor(variables, dtype=torch.int64, device=dev), per)
    out = torch.empty((count, 3), dtype=torch.int64, device=dev)
    out[:, 0] = var
    out[:, 1] = sets[:count]
    out[:, 2] = scores[:count].view(torch.int32).to(torch.int64)
    return out


def allgather_lists(packed: torch.Tensor, world_size: int, group=None) -> torch.Tensor:
    """One all-gather of variable-length [count, 3] blocks (counts first, then
    the blocks padded to the largest); returns the concatenation in rank order."""
    return allgather_rows(packed, world_size, group)


def allgather_rows(packed: torch.Tensor, world_size: int, group=None) -> torch.Tensor:
    """allgather_lists for int64 rows of any width."""
    dev = packed.device
    w = packed.shape[1]
    cnt = torch.tensor([packed.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world_size)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(max(counts), 1)
    buf = torch.zeros((mx, w), dtype=torch.int64, device=dev)
    buf[: packed.shape[0]] = packed
    out = torch.empty((world_size * mx, w), dtype=torch.int64, device=dev)
    if hasattr(dist, "all_gather_into_tensor") and dev.type != "cpu":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        parts = [torch.empty_like(buf) for _ in range(world_size)]
        dist.all_gather(parts, buf, group=group)
        out = torch.cat(parts, 0)
    keep = torch.cat([torch.arange(r * mx, r * mx + counts[r], device=dev) for r in range(world_size)])
    return out[keep]


def unpack(gathered: torch.Tensor, n: int):
    """-> (offsets[n+1], sets uint64, scores float32) in variable order; the
    order inside a variable is the order its owning rank produced."""
    g = gathered.cpu().numpy()
    order = np.argsort(g[:, 0], kind="stable")
    g = g[order]
    counts = np.bincount(g[:, 0], minlength=n)
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(counts)
    sets = g[:, 1].view(np.uint64).copy()
    scores = g[:, 2].astype(np.int32).view(np.float32).copy()
    return offsets, sets, scores


# ---- triplet_astar clusters -------------------------------------------------

def assign_clusters(clusters, world_size: int) -> np.ndarray:
    """Owner rank per cluster: longest-processing-time first, a cluster of c
    variables priced at 2^c (the order lattice its A* may expand), ties to the
    lower rank; deterministic, so every rank computes the same split."""
    sizes = [bin(int(c)).count("1") for c in clusters]
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    loads = [0] * world_size
    owner = np.zeros(len(sizes), dtype=np.int64)
    for i in order:
        r = min(range(world_size), key=lambda q: (loads[q], q))
        owner[i] = r
        loads[r] += 1 << sizes[i]
    return owner


def pack_memo(clusters, parents, n: int, device="cpu") -> torch.Tensor:
    """[k, 1 + n] int64 rows: cluster, then each variable's parent set (uint64 bits)."""
    k = len(clusters)
    out = np.zeros((k, 1 + n), dtype=np.int64)
    if k:
        out[:, 0] = np.asarray(clusters, dtype=np.uint64).view(np.int64)
        out[:, 1:] = np.asarray(parents, dtype=np.uint64).reshape(k, n).view(np.int64)
    return torch.from_numpy(out).to(device)


def unpack_memo(gathered: torch.Tensor):
    g = gathered.cpu().numpy()
    return g[:, 0].view(np.uint64).copy(), g[:, 1:].view(np.uint64).copy()


def triplet_sharded(ctx, edges, world_size: int, rank: int, pd_count: int = 2, group=None, device="cpu"):
    """ulg_triplet_astar over world_size ranks (one libulg context each, same
    lists loaded): the first sweep's clusters solved once each across ranks,
    one all-gather, then the driver on every rank.  Returns ctx.triplet()'s
    dict plus "solved_here" (clusters this rank searched before the exchange)
    and "expanded_here"."""
    n = ctx.search_n
    clusters = ctx.triplet_clusters(edges)
    if world_size == 1:  # nothing to share: the driver alone searches only what it asks for
        res = ctx.triplet(edges=edges, pd_count=pd_count)
        res.update(solved_here=0, expanded_here=0, clusters=len(clusters))
        return res
    owner = assign_clusters(clusters, world_size)
    mine = clusters[owner == rank]
    parents, st = ctx.triplet_solve(mine, pd_count)
    gathered = allgather_rows(pack_memo(mine, parents, n, device), world_size, group)
    cl, pa = unpack_memo(gathered)
    ctx.triplet_memo_put(cl, pa, pd_count)
    res = ctx.triplet(edges=edges, pd_count=pd_count)
    res["solved_here"] = st["distinct"]
    res["expanded_here"] = st["expanded"]
    res["clusters"] = len(clusters)
    return res
