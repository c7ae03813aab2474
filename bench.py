#!/usr/bin/env python3
"""Benchmark of the MI355X cBIC-score hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2] [--mode weak|shard]

One step = one full cBIC scoring pass (every parent set of size <= k of every
variable through the layer-synchronous HIP scorer, stored-set rule and
dominance recursion included) over inputs already resident in HBM.

--mode weak (default): every rank scores the whole configuration on its own
    synthetic dataset (seed 9200 + rank): a batch of independent structure-
    learning problems, per-GPU work fixed as N grows, no collective in the
    data path.
--mode shard: one dataset, variables striped over ranks (score_main.cpp:136-139)
    and the per-variable (set, score) lists exchanged with one RCCL
    all_gather inside the timed step; strong scaling.

Rank 0 prints one JSON line.  cpu_baseline = the CPU oracle (a faithful C
restatement that solves each OLS over all N rows like the reference) timed on
a bounded sample on this host, rank 0 at N=1 only.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))

import shard  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402

METRIC = "cBIC parent-set scores/sec + A* expansions/sec, n=25 full skeleton"
CONFIGS = {
    "c2": dict(n=20, N=10000, k=4, lam=2.0),
    "c3": dict(n=25, N=10000, k=6, lam=2.0),
    # BASELINE C4: n=30, N=100k, MMPC skeleton (built on the GPU from the same
    # data, alpha 0.01), 2-hop candidate sets; k capped at the HIP scorer's 8
    "c4": dict(n=30, N=100000, k=8, lam=2.0, skeleton="mmpc", alpha=0.01),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def cpu_baseline(cfg, X, target_s=15.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    n, k, lam = cfg["n"], cfg["k"], cfg["lam"]
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1))
    nvars = min(n, threads)
    variables = list(range(nvars))
    cands = [(1 << n) - 1] * n
    ds = oracle.Dataset(X)
    t0 = time.perf_counter()
    probe_frac = 0.002
    c0 = oracle.score_sample(ds, lam, variables, cands, k, probe_frac, threads)
    dt0 = time.perf_counter() - t0
    frac = min(1.0, probe_frac * target_s / max(dt0, 1e-3))
    t0 = time.perf_counter()
    c = oracle.score_sample(ds, lam, variables, cands, k, frac, threads)
    dt = time.perf_counter() - t0
    return {"value": c / dt, "unit": "parent-set scores/s", "cores": threads, "kind": "port",
            "sample": f"CPU oracle (C restatement, per-set OLS over all N rows) on {nvars} of {n} variables, "
                      f"first {frac:.4f} of every layer 1..{k} in Gosper order: {c} parent sets in {dt:.2f} s "
                      f"on {threads} threads"}


PMC_TRAFFIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r1", "pmc_traffic.json")


def pmc_traffic(cfg, sets, label):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    PMC passes of the same config (scripts/pmc_round.sh + pmc_summarize.py);
    None if there is no summary for this config and launch size."""
    try:
        t = json.load(open(PMC_TRAFFIC))
    except (OSError, ValueError):
        return None, None
    if (t.get("config_id") != cfg["id"] or round(t.get("sets_per_launch", -1)) != round(sets)
            or t.get("label") != label):
        return None, None
    return t["traffic_bytes_per_launch"], "profiles/r1/pmc_traffic.json"


def roofline(ctx, cfg, per_layer_sets, steps):
    """Dominant unit = the layer-k 'rest' launch (sets without variable 0): the
    scoring kernel plus, with the two-pass scorer (score_variant bit 4), the
    walk kernel over the sets it queued -- both are one layer's decision, so
    their average durations are summed (rocprof lists them separately)."""
    k = cfg["k"]
    names = [f"score_layer_{k}_rest", f"walk_{k}_rest"]
    ps = [ctx.profile_get(nm) for nm in names]
    if ps[0] is None:
        return None, None
    if ps[1] is None:
        names, ps = names[:1], ps[:1]
    name = " + ".join(names)
    p = {"avg_ms": sum(q["avg_ms"] for q in ps), "count": ps[0]["count"]}
    # the scorer stripes the variables over concurrent stream groups
    # (score_streams): one launch covers 1/groups of the layer's sets
    groups = max(1, round(ps[0]["count"] / steps))
    sets = per_layer_sets / groups
    # compulsory HBM bytes per scored set = 4 (k direct-subset score reads) + 4 (score write)
    bytes_per_set = 4 * (k + 1)
    achieved = sets * bytes_per_set / (p["avg_ms"] * 1e-3) / 1e9
    flops_per_set = 2 * k ** 3 / 3 + 2 * k * k + 2 * k
    traffic, traffic_src = pmc_traffic(cfg, sets, name)
    return ({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per launch",
             "traffic_source": traffic_src, "kernel": name,
             "avg_launch_ms": p["avg_ms"], "avg_launch_ms_each": [q["avg_ms"] for q in ps],
             "launches": p["count"], "launches_per_step": groups, "sets_per_launch": sets,
             "note": "launches of different stream groups overlap; each duration is its own kernel's",
             "bytes_per_set": bytes_per_set,
             "fp64_flops_per_set": flops_per_set,
             "fp64_tflops": sets * flops_per_set / (p["avg_ms"] * 1e-3) / 1e12}, p)


PMC_SEARCH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r1", "pmc_search_traffic.json")


def search_roofline(cfg, n, pull, reps):
    """Roofline of the GPU order-graph sweep (layer_pull_kernel, one launch
    per layer) on a full skeleton: a layer-L node reads L predecessors' g
    (4 B) and best-score keys (8 B) and writes its g (4 B) and leaf (1 B), so
    one sweep's algorithmic bytes are sum_L C(n, L) (12 L + 5).  The achieved
    rate divides them by the sweep's summed kernel time (HIP events on the
    launch stream); traffic is the PMC-measured bytes of one sweep."""
    cnt, sweep_ms = pull["count"], pull["total_ms"] / reps
    algo = sum(math.comb(n, L) * (12 * L + 5) for L in range(1, n + 1))
    achieved = algo / (sweep_ms * 1e-3) / 1e9
    traffic, src = None, None
    try:
        t = json.load(open(PMC_SEARCH))
        if t.get("config_id") == cfg["id"] and t.get("n") == n:
            traffic, src = t["traffic_bytes_per_sweep"], "profiles/r1/pmc_search_traffic.json"
    except (OSError, ValueError):
        pass
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per sweep",
            "traffic_source": src, "kernel": "layer_pull_kernel", "launches_per_sweep": cnt // reps,
            "sweep_kernel_ms": sweep_ms, "algorithmic_bytes_per_sweep": algo,
            "bytes_per_node": "12 L + 5 (L predecessors x (4 B g + 8 B key) + 4 B g + 1 B leaf written)"}


def search_metrics(ctx, cfg, variables, cands, rank, ws, reps=3, edges=None, skel_note="full skeleton"):
    """Order-graph search side on this rank's scored lists: GPU best-score
    tables + pattern database + GPU layer-synchronous search at the bench
    config (A* expansions/s), then the exact-order A* (reference pop order,
    bit-exact DAG) and the CPU oracle's A* on config C2 (rank 0, N=1 only)."""
    import time as _t
    n, k = cfg["n"], cfg["k"]
    full = [(1 << n) - 1] * n
    skel = full if edges is None else edges
    out = {}
    ctx.score(list(range(n)), full if edges is None else ulg.candidates_from_edges(edges, n), k)
    t0 = _t.perf_counter()
    ctx.search_from_scores()
    t1 = _t.perf_counter()
    tables_ms = 1e3 * (t1 - t0)
    ctx.search_from_scores()  # again, with the 3.4 GB of C3 tables already allocated
    tables_again_ms = 1e3 * (_t.perf_counter() - t1)
    t1 = _t.perf_counter()
    ctx.pdb_build(2)
    t2 = _t.perf_counter()
    best = None
    # HIP events around every layer_pull_kernel launch of the sweeps
    ctx.profile(True)
    ctx.profile_select(["search_layer_pull"])
    ctx.profile_reset()
    for _ in range(reps):
        ts = _t.perf_counter()
        g = ctx.astar(edges=skel, mode=1, net_text=False)
        dt = _t.perf_counter() - ts
        best = dt if best is None else min(best, dt)
    pull = ctx.profile_get("search_layer_pull")
    ctx.profile(False)
    out["gpu_search"] = {"config": f"{cfg['id'].upper()} lists (n={n}, k={k}), {skel_note}, static PDB(2)",
                         "expansions": g["expanded"], "ms": 1e3 * best,
                         "expansions_per_s": g["expanded"] / best, "goal_cost": g["cost"],
                         "tables_ms": tables_ms, "tables_rebuild_ms": tables_again_ms,
                         "pdb_ms": 1e3 * (t2 - t1),
                         "note": "layer-synchronous pull over the whole order lattice; best of %d" % reps}
    if edges is None and pull is not None:
        out["gpu_search"]["roofline"] = search_roofline(cfg, n, pull, reps)
    if rank == 0 and ws == 1:
        c2 = CONFIGS["c2"]
        n2, N2, k2 = c2["n"], c2["N"], c2["k"]
        X2, _ = synth.gaussian_sem(n2, N2, 9200)
        full2 = [(1 << n2) - 1] * n2
        ctx.load(X2, c2["lam"])
        ctx.score(list(range(n2)), full2, k2)
        ctx.search_from_scores()
        ts = _t.perf_counter()
        e = ctx.astar(edges=full2, mode=0, net_text=False)
        dt = _t.perf_counter() - ts
        out["exact"] = {"config": f"C2 (n={n2}, N={N2}, k={k2}), full skeleton", "expansions": e["expanded"],
                        "ms": 1e3 * dt, "expansions_per_s": e["expanded"] / dt, "goal_cost": e["cost"],
                        "note": "reference pop order replayed on the host over GPU-built O(1) tables (incl. table D2H)"}
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        offs, sets, scores = ctx.fetch(ctx.score(list(range(n2)), full2, k2)[0])
        costs = ctx.quantize(scores)
        srch = oracle.Search(n2, offs, sets, costs)
        ts = _t.perf_counter()
        r = srch.astar(edges=full2)
        dt = _t.perf_counter() - ts
        out["cpu_baseline"] = {"value": r["expanded"] / dt, "unit": "A* expansions/s", "cores": 1, "kind": "port",
                               "sample": f"CPU oracle A* (sorted-list scans, reference heap) on C2: "
                                         f"{r['expanded']} expansions in {dt:.2f} s",
                               "same_dag_as_exact": [int(x) for x in r["vpar"]] == [int(x) for x in e["vpar"]]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="weak", choices=["weak", "shard"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-search", action="store_true")
    ap.add_argument("--score-variant", type=int, default=None, help="A/B knob (ulg_set_option score_variant)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + --device: rehearse the N>1 code path with several ranks on one GPU")
    ap.add_argument("--device", type=int, default=None, help="GPU for every rank (default LOCAL_RANK)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    cfg = dict(CONFIGS[args.config], id=args.config)
    n, N, k, lam = cfg["n"], cfg["N"], cfg["k"], cfg["lam"]

    import torch
    dist = None
    if args.device is not None:
        local = args.device
    cdev = "cuda" if args.dist_backend == "nccl" else "cpu"  # where collective tensors live
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend, rank=rank, world_size=ws)

    seed = 9200 + (rank if args.mode == "weak" else 0)
    X, _ = synth.gaussian_sem(n, N, seed)
    ctx = ulg.Context(local)
    if args.score_variant is not None:
        ctx.set_option("score_variant", args.score_variant)
    ctx.load(X, lam)
    cands_all = [(1 << n) - 1] * n
    skel_note = "full n x n skeleton"
    if cfg.get("skeleton") == "mmpc":
        rows = ctx.mmpc(cfg["alpha"])
        cands_all = ulg.candidates_from_edges(rows, n)
        skel_note = (f"MMPC skeleton (ulg_mmpc, alpha {cfg['alpha']}: {sum(bin(r).count('1') for r in rows) // 2} "
                     f"edges), 2-hop candidate sets")
    if args.mode == "shard":
        variables = shard.stripe(n, ws, rank)
    else:
        variables = list(range(n))
    cands = [cands_all[v] for v in variables]
    msz = [bin(cands_all[v] & ~(1 << v)).count("1") for v in range(n)]
    units_rank = sum(sum(math.comb(msz[v], L) for L in range(k + 1)) for v in variables)

    def step():
        stored, scored = ctx.score(variables, cands, k)
        if args.mode == "shard" and ws > 1:
            # one RCCL all-gather of the per-variable (set, score) lists (shard.py)
            sets_t = torch.empty(max(stored, 1), dtype=torch.int64, device="cuda")
            sc_t = torch.empty(max(stored, 1), dtype=torch.float32, device="cuda")
            off_t = torch.empty(len(variables) + 1, dtype=torch.int64, device="cuda")
            ctx.fetch_device(sets_t.data_ptr(), sc_t.data_ptr(), off_t.data_ptr())
            shard.allgather_lists(shard.pack_device(variables, off_t, sets_t, sc_t).to(cdev), ws)
        return scored

    for _ in range(args.warmup):
        step()
    # HIP events in the timed region only around the roofline unit's kernels
    # (two host-side event records per timed kernel would otherwise show up in
    # a ~2 ms step of ~35 launches); the full per-kernel breakdown comes from
    # one extra profiled step after the timed region
    ctx.profile(True)
    ctx.profile_select([f"score_layer_{k}_rest", f"walk_{k}_rest"])
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scored_total = 0
    for _ in range(args.steps):
        scored_total += step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.profile(False)
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        u = torch.tensor([scored_total], dtype=torch.float64, device=cdev)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        scored_all = float(u.item())
    else:
        scored_all = float(scored_total)

    # sets in one launch of the dominant kernel (layer k, sets without variable 0)
    per_launch = sum(math.comb(msz[v] - (1 if (v != 0 and cands_all[v] & 1) else 0), k) for v in variables)
    roof, _ = roofline(ctx, cfg, per_launch, args.steps)
    ctx.profile(True)
    ctx.profile_select(None)
    ctx.profile_reset()
    step()
    kernels = ctx.profile_dump()
    ctx.profile(False)

    search = None
    if args.mode == "weak" and not args.no_search:
        search = search_metrics(ctx, cfg, variables, cands, rank, ws,
                                edges=rows if cfg.get("skeleton") == "mmpc" else None, skel_note=skel_note)

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": scored_all / elapsed,
            "unit": "parent-set scores/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "weak" else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: seeded linear-Gaussian SEM (synth.gaussian_sem, seed "
                    f"{'9200+rank' if args.mode == 'weak' else '9200, one dataset'}), {skel_note}",
            "config": {"workload": f"{args.config.upper()} cBIC scoring: n={n}, N={N}, max-parents k={k}, "
                                   f"lambda={lam}, {skel_note}, all {n} variables per "
                                   f"{'GPU' if args.mode == 'weak' else 'job'}",
                       "config_id": args.config, "mode": args.mode,
                       "parent_sets_per_step_per_rank": units_rank},
            "roofline": roof,
            "kernel_ms_one_step": {kk: round(vv["total_ms"], 4) for kk, vv in kernels.items()},
        }
        if search is not None:
            res["astar"] = search
        if ws == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg, X)
        print(json.dumps(res))
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
