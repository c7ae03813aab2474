"""Variable-sharded scoring across ranks (one process per GPU) and the single
exchange step of SURVEY 8e: every rank scores its stripe of the variables
(v % world_size == rank, as score_main.cpp:136-139 stripes threads), then one
all-gather (RCCL over xGMI on MI355X; gloo in the CPU tests) hands every rank
the complete per-variable (set, score) lists in variable order, ready for
ulg_search_load or a .pss writer.

Wire format per entry: int64 [variable, set, float32 score bits]."""
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
    dev = packed.device
    cnt = torch.tensor([packed.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world_size)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(max(counts), 1)
    buf = torch.zeros((mx, 3), dtype=torch.int64, device=dev)
    buf[: packed.shape[0]] = packed
    out = torch.empty((world_size * mx, 3), dtype=torch.int64, device=dev)
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
