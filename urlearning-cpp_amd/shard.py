"""Variable-sharded scoring across ranks (one process per GPU) and the single
exchange step of SURVEY 8e.

Scoring.  Every variable has its own cache and dominance check
(score_main.cpp:143-155; the reference's threads stripe variables,
:136-139), so ranks score disjoint variable sets with no communication.
`assign` balances them by the parent sets each variable scores,
sum_{L<=k} C(m_v, L) with m_v = |candidates(v) \ {v}|, longest
first.  `ListExchange` then runs the ONE collective of the data path: an
all-gather (RCCL over xGMI on MI355X; gloo in the CPU tests) of fixed-size
per-rank blocks.  A block holds the rank's local offsets followed by its
stored sets and scores, written straight from the scorer's device buffers
(ulg_cbic_fetch with device pointers).  The first exchange sizes the blocks
by the a-priori bound "every scored set is stored", which every rank
computes from (candidates, k), so no count exchange precedes the data; the
headers carry the counts, and later exchanges use the learned capacity
(ListExchange).  After the gather every rank holds
every variable's list in variable order, ready for ulg_search_load_scores
(local best-score tables + search) or a .pss writer.

triplet_astar shards the same way: its distinct clusters are
independent exact A* problems (triplet_astar.cpp:285-674, one per cluster).
Every rank enumerates the first sweep's clusters (ulg_triplet_clusters),
solves its share (ulg_triplet_solve), one all-gather of [cluster, parents...]
rows fills every rank's memo (ulg_triplet_memo_put), and the sequential
driver (ulg_triplet_astar) then runs on each rank with nothing left to search
but the clusters that orientations add mid-sweep -- the MEC is the one a
single GPU computes.  (That exchange is off the scoring path and sends a
count first: allgather_rows.)"""
from __future__ import annotations

from math import comb

import numpy as np
import torch
import torch.distributed as dist


def stripe(n: int, world_size: int, rank: int):
    """The reference's thread striping (score_main.cpp:136-139): v % T."""
    return [v for v in range(n) if v % world_size == rank]


def var_weight(n: int, v: int, candidates: int, k: int) -> int:
    """Parent sets the scorer evaluates for v: sum_{L<=k} C(m_v, L), the
    empty set included (score_calculator.cpp:54-120)."""
    m = bin(int(candidates) & ~(1 << v) & ((1 << n) - 1)).count("1")
    kk = m if k < 1 or k > m else k
    return sum(comb(m, L) for L in range(kk + 1))


def assign(n: int, world_size: int, candidates, k: int):
    """Deterministic balanced partition of the variables over ranks:
    longest-processing-time first on var_weight (ties: lower variable, lower
    rank).  Returns one ascending variable list per rank."""
    w = [var_weight(n, v, candidates[v], k) for v in range(n)]
    order = sorted(range(n), key=lambda v: (-w[v], v))
    loads = [0] * world_size
    parts = [[] for _ in range(world_size)]
    for v in order:
        r = min(range(world_size), key=lambda q: (loads[q], q))
        parts[r].append(v)
        loads[r] += w[v]
    return [sorted(p) for p in parts]


def table_owners(n: int, world_size: int, candidates=None):
    """Variables whose best-score tables and sweep slices each rank holds in
    the variable-sharded sweep (n >= 31): longest-processing-time
    on the table size 2^{m_v} (every variable's is 2^{n-1} on a full
    skeleton, so this is a balanced stripe).  Returns one bit mask per rank."""
    cands = candidates if candidates is not None else [(1 << n) - 1] * n
    w = [1 << bin(int(cands[v]) & ~(1 << v) & ((1 << n) - 1)).count("1") for v in range(n)]
    order = sorted(range(n), key=lambda v: (-w[v], v))
    loads = [0] * world_size
    masks = [0] * world_size
    for v in order:
        r = min(range(world_size), key=lambda q: (loads[q], q))
        masks[r] |= 1 << v
        loads[r] += w[v]
    return masks


def sharded_sweep(ctx, n: int, own: int, device="cuda", comm_device=None, keys=None):
    """The GPU order-graph sweep with the tables sharded by variable
    (ulg_sweep_shard_*): per layer this rank's best (cost, leaf) keys over the
    leaves it owns, ONE MIN all-reduce of the layer's keys over the ranks
    (RCCL over xGMI; gloo copies through the host), then the commit.  Every
    rank returns the single-GPU ULG_ASTAR_GPU result.  `keys`: a reusable
    int64 device buffer of at least the largest layer."""
    comm_device = comm_device or device
    maxl = ctx.sweep_shard_begin(own)
    if keys is None or keys.numel() < maxl:
        keys = torch.empty(maxl, dtype=torch.int64, device=device)
    stage = torch.empty(maxl, dtype=torch.int64, device=comm_device) if comm_device != device else None
    for L in range(1, n + 1):
        cnt = comb(n, L)
        view = keys[:cnt]
        ctx.sweep_shard_layer(L, view.data_ptr())  # synchronised: the keys are complete
        if dist.is_initialized() and dist.get_world_size() > 1:
            if stage is None:
                dist.all_reduce(view, op=dist.ReduceOp.MIN)
                torch.cuda.synchronize()
            else:
                st = stage[:cnt]
                st.copy_(view)
                dist.all_reduce(st, op=dist.ReduceOp.MIN)
                view.copy_(st)
                torch.cuda.synchronize()
        ctx.sweep_shard_commit(L, view.data_ptr())
    return ctx.sweep_shard_end()


class ListExchange:
    """One all-gather of every rank's stored (set, score) lists.

    Block layout (bytes; every rank computes the same sizes):
      [0, hdr)                   int64 local offsets[nv_r + 1] (ulg_cbic_fetch)
      [hdr, hdr + w cap)         stored sets: uint32 when n <= 32 (w = 4), else uint64 (w = 8)
      [hdr + w cap, + 4 cap)     float32 scores
    With n <= 32 a set is its low 32 bits, so the block carries 8 B per set
    instead of 12; the sets are fetched into a staging buffer and narrowed on
    the device.

    Capacity.  The first exchange uses the a-priori bound "every scored set
    stored" (max over ranks of sum_{v in rank} var_weight), which needs no
    count exchange.  Every block's header carries its rank's stored count, so
    after each gather every rank knows every count and the next exchanges use
    a learned capacity: the largest count plus `slack` (at C3 the stored lists
    are a third of the scored sets, so the blocks shrink about 3x).  A rank
    whose lists outgrow the capacity sends its header only; every rank sees
    that in the gathered headers, all grow the capacity to the largest count
    and gather once more (a second collective only then)."""

    def __init__(self, n: int, parts, candidates, k: int, rank: int, device="cuda", comm_device=None,
                 learn=True, slack=0.02):
        self.n, self.parts, self.rank, self.ws = n, parts, rank, len(parts)
        self.mine = parts[rank]
        bounds = [sum(var_weight(n, v, candidates[v], k) for v in p) for p in parts]
        self.bound = max(max(bounds), 1)  # the a-priori capacity
        self.learn, self.slack = learn, slack
        maxnv = max(len(p) for p in parts)
        self.narrow = n <= 32
        self.w = 4 if self.narrow else 8
        self.hdr = 16 * ((8 * (maxnv + 1) + 15) // 16)
        self.device = torch.device(device)
        self.comm_device = torch.device(comm_device) if comm_device is not None else self.device
        self.regathers = 0  # exchanges that had to grow the capacity and gather again
        self.counts = None  # every rank's stored count at the last gather
        self._src = None
        self._next = None  # learned capacity, adopted by the next fill
        self._resize(self.bound)

    def _resize(self, cap: int):
        self.cap = max(int(cap), 1)
        self.block = 16 * ((self.hdr + (self.w + 4) * self.cap + 15) // 16)
        self.buf = torch.zeros(self.block, dtype=torch.uint8, device=self.device)
        self.out = torch.empty(self.ws * self.block, dtype=torch.uint8, device=self.comm_device)
        base = self.buf.data_ptr()
        self.offs_ptr = base
        self.scores_ptr = base + self.hdr + self.w * self.cap
        if self.narrow:
            self.stage = torch.zeros(self.cap, dtype=torch.int64, device=self.device)
            self.sets_ptr = self.stage.data_ptr()
        else:
            self.sets_ptr = base + self.hdr
        self._fills_done = None
        if self.device.type == "cuda":
            # the zero fills run on torch's stream and libulg writes these
            # blocks on its own (ulg.h's stream contract: ulg_cbic_fetch is not
            # ordered after other streams' work): the next fetch makes the
            # context's stream wait for this event, so no fill can land after
            # the scorer's copy and zero the lists
            self._fills_done = torch.cuda.Event()
            self._fills_done.record(torch.cuda.current_stream(self.device))

    def _sets_view(self, blocks):
        """[ws, cap] int64 sets of gathered blocks [ws, block] (uint8)."""
        raw = blocks[:, self.hdr:self.hdr + self.w * self.cap].contiguous()
        if not self.narrow:
            return raw.view(torch.int64)
        return raw.view(torch.int32).to(torch.int64) & 0xFFFFFFFF

    def _write(self):
        """Fill the send block from the remembered source (header only when
        the lists do not fit)."""
        kind, a, b = self._src
        if kind == "ctx":
            ctx, stored = a, b
            if self._fills_done is not None:
                ctx.stream_wait_event(self._fills_done)
                self._fills_done = None
            if stored <= self.cap:
                ctx.fetch_device(self.sets_ptr, self.scores_ptr, self.offs_ptr)
                if self.narrow:
                    # low 32 bits of each set (little endian), on the device
                    lo = self.stage.view(torch.int32).view(-1, 2)[:, 0]
                    self.buf[self.hdr:self.hdr + 4 * self.cap].view(torch.int32).copy_(lo)
            else:  # header only: just the offsets (null sets / scores pointers skip those copies)
                ctx.fetch_device(0, 0, self.offs_ptr)
            return
        offsets, sets, scores = a
        cnt = int(offsets[-1])
        b = np.zeros(self.block, dtype=np.uint8)
        b[:8 * len(offsets)] = offsets.view(np.uint8)
        if cnt <= self.cap:
            st = np.asarray(sets[:cnt], dtype=np.uint64)
            if self.narrow:
                if cnt and int(st.max()) >> 32:
                    raise RuntimeError("shard: a set above bit 31 with n <= 32")
                st = st.astype(np.uint32)
            b[self.hdr:self.hdr + self.w * cnt] = st.view(np.uint8)
            o = self.hdr + self.w * self.cap
            b[o:o + 4 * cnt] = np.asarray(scores[:cnt], dtype=np.float32).view(np.uint8)
        self.buf.copy_(torch.from_numpy(b))

    def _adopt(self):
        # the learned capacity replaces the blocks (the previous gather's
        # output is no longer needed once the next fill starts)
        if self._next is not None and self._next < self.cap:
            self._resize(self._next)
        self._next = None

    def fill(self, ctx, stored: int):
        """Write this rank's lists (the last ctx.score over self.mine) into
        the send block, straight from the scorer's device buffers."""
        self._adopt()
        self._src = ("ctx", ctx, int(stored))
        self._write()

    def fill_host(self, offsets, sets, scores):
        """Same from host lists (local offsets[nv_r + 1], sets, scores), e.g.
        the CPU oracle's in the gloo tests."""
        self._adopt()
        offsets = np.asarray(offsets, dtype=np.int64)
        self._src = ("host", (offsets, sets, scores), None)
        self._write()

    def _gather(self, group):
        src = self.buf if self.comm_device == self.device else self.buf.to(self.comm_device)
        if self.comm_device.type != "cpu":
            dist.all_gather_into_tensor(self.out, src, group=group)
        else:
            parts = list(self.out.view(self.ws, self.block).unbind(0))
            dist.all_gather(parts, src, group=group)

    def _read_counts(self):
        hdr = self.out.view(self.ws, self.block)[:, :self.hdr].cpu().numpy().view(np.int64)
        return [int(hdr[r, len(p)]) for r, p in enumerate(self.parts)]

    def allgather(self, group=None):
        """The data-path collective: one all-gather of fixed-size blocks
        (a second one only if some rank's lists outgrew the capacity)."""
        self._gather(group)
        self.counts = self._read_counts()  # one small D2H of the headers
        need = max(self.counts)
        if need > self.cap:
            self.regathers += 1
            self._resize(need + int(self.slack * need) + 256)
            self._write()
            self._gather(group)
            self.counts = self._read_counts()
        self._next = need + int(self.slack * need) + 256 if self.learn else None
        return self.out

    def assemble(self, device=None):
        """-> (offsets[n+1] int64 numpy, sets int64 tensor, scores float32
        tensor) in variable order, on `device` (default: where the gathered
        blocks are)."""
        dev = torch.device(device) if device is not None else self.out.device
        blocks = self.out.view(self.ws, self.block)
        hdr = blocks[:, :self.hdr].cpu().numpy().view(np.int64)  # one small D2H of the headers
        src = blocks.to(dev) if blocks.device != dev else blocks
        sets_all = self._sets_view(src)  # [ws, cap]
        so = self.hdr + self.w * self.cap
        scores_all = src[:, so:so + 4 * self.cap].contiguous().view(torch.float32)
        where = {}
        for r, p in enumerate(self.parts):
            for i, v in enumerate(p):
                where[v] = (r, int(hdr[r, i]), int(hdr[r, i + 1]))
        offsets = np.zeros(self.n + 1, dtype=np.int64)
        idx = []
        for v in range(self.n):
            r, b, e = where[v]
            offsets[v + 1] = offsets[v] + (e - b)
            idx.append(torch.arange(r * self.cap + b, r * self.cap + e, dtype=torch.int64))
        gi = torch.cat(idx).to(dev) if idx else torch.zeros(0, dtype=torch.int64, device=dev)
        sets, scores = sets_all.reshape(-1)[gi], scores_all.reshape(-1)[gi]
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)  # libulg reads them on its own stream
        return offsets, sets, scores


def allgather_rows(packed: torch.Tensor, world_size: int, group=None) -> torch.Tensor:
    """All-gather of variable-length int64 [count, w] blocks (counts first,
    then the blocks padded to the largest); the concatenation in rank order."""
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
