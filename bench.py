#!/usr/bin/env python3
"""Benchmark of the MI355X cBIC-score hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4] [--mode shard|weak]

One step = one full cBIC scoring pass over one dataset (every parent set of
size <= k of every variable through the layer-synchronous HIP scorer,
stored-set rule and dominance recursion included) over inputs already
resident in HBM.

--mode shard (default): SURVEY 8e.  The variables are balanced over the
    ranks by the parent sets each one scores (shard.assign), every rank
    scores its share, and the per-variable (set, score) lists are exchanged
    with ONE all-gather (RCCL over xGMI) inside the timed step
    (shard.ListExchange).  After the timed region every rank builds its own
    best-score tables and pattern database from the gathered lists and runs
    the GPU order-graph search (A* is replicas-only); the exchange,
    table build and search are reported separately.  Strong scaling: the
    job's work is fixed as N grows.  At N = 1 there is no exchange.
--mode weak: every rank scores the whole configuration on its own synthetic
    dataset (seed 9200 + rank), no collective in the data path.

--gpus N > 1 without WORLD_SIZE in the environment starts N worker processes
(one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1 set) before
anything touches the GPU and exits with their status; under
torch.distributed.run the ranks come from the environment and --gpus must
agree with WORLD_SIZE.

Rank 0 prints one JSON line.  cpu_baseline = the CPU oracle (a faithful C
restatement that solves each OLS over all N rows like the reference) timed on
a bounded sample on this host, rank 0 at N=1 only.
"""
import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
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
    # data, alpha 0.01), 2-hop candidate sets, the reference's default parent
    # limit -p = n - 1 (score_main.cpp:296-298): layers 9..18 run the wide kernels
    "c4": dict(n=30, N=100000, k=29, lam=2.0, skeleton="mmpc", alpha=0.01),
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
    # the CPUs this process may actually use: its affinity mask, capped by the
    # cgroup CPU quota (on the GPU box 16 of 256 visible CPUs); more threads
    # than that only time-share them
    cores = max(1, len(os.sched_getaffinity(0)))
    q = cpu_quota()
    if q is not None:
        cores = max(1, min(cores, int(q)))
    threads = cores
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
    return {"value": c / dt, "unit": "parent-set scores/s", "cores": cores, "threads": threads, "kind": "port",
            "cpu": cpu_model(), "cpu_quota": q, "affinity_cpus": len(os.sched_getaffinity(0)),
            "sample": f"CPU oracle (C restatement, per-set OLS over all N rows) on {nvars} of {n} variables, "
                      f"first {frac:.4f} of every layer 1..{k} in Gosper order: {c} parent sets in {dt:.2f} s "
                      f"on {threads} threads"}


PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r2")
# the scorer's counter passes of this round's kernels (scripts/gpu_probe.sh
# step pmc_scorer + pmc_r5_summarize.py on the same bench command)
PMC_SCORER = os.path.join(os.path.dirname(PROFILES), "r6", "pmc_scorer.json")


def pmc_scorer(cfg, sets, label):
    """Counters of the roofline pair from the committed rocprofv3 PMC passes
    of the same config and launch size: HBM traffic per launch (2 x FETCH_SIZE
    + WRITE_SIZE), vector-L1 line lookups per set and the TA busy fraction.
    None when there is no summary for this config, launch and kernel pair."""
    try:
        t = json.load(open(PMC_SCORER))
    except (OSError, ValueError):
        return None
    if (t.get("config_id") != cfg["id"] or round(t.get("sets_per_launch", -1)) != round(sets)
            or t.get("label") != label):
        return None
    return t


ROOF_KERNELS = ["score_layer_{k}_rest", "walk_{k}_rest"]


def roofline(ctx, cfg, per_layer_sets, steps):
    """Dominant unit: the layer-k 'rest' launch (sets without variable 0):
    the scoring kernel plus, with the two-pass scorer (score_variant bit 4),
    the walk kernel over the sets it queued -- both are one layer's decision,
    so their average durations are summed (rocprof lists them separately)."""
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
    pmc = pmc_scorer(cfg, sets, name)
    traffic = pmc["traffic_bytes_per_launch"] if pmc else None
    return ({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per launch",
             "traffic_source": os.path.relpath(PMC_SCORER, ROOT) if pmc else None,
             "l1_lines_per_set": pmc.get("l1_lines_per_set") if pmc else None,
             "ta_busy_frac": pmc.get("ta_busy_frac") if pmc else None,
             "score_valu_per_wave": pmc.get("score", {}).get("valu_per_wave") if pmc else None,
             "score_resident_waves_per_simd": pmc.get("score", {}).get("resident_waves_per_simd") if pmc else None,
             "pmc_kernels": pmc.get("kernels") if pmc else None,
             "pmc_note": ("what binds the pair is the vector memory pipeline, not HBM bytes: l1_lines_per_set = "
                          "TCP_TOTAL_CACHE_ACCESSES / sets (one tag lookup per distinct 128-B line per gather "
                          "instruction), ta_busy_frac = per-CU TA_TA_BUSY / kernel cycles of the scoring kernel "
                          "(profiles/r6, scripts/pmc_r5_summarize.py)"),
             "kernel": name,
             "avg_launch_ms": p["avg_ms"], "avg_launch_ms_each": [q["avg_ms"] for q in ps],
             "launches": p["count"], "launches_per_step": groups, "sets_per_launch": sets,
             "note": "launches of different stream groups overlap; each duration is its own kernel's",
             "bytes_per_set": bytes_per_set,
             "fp64_flops_per_set": flops_per_set,
             "fp64_tflops": sets * flops_per_set / (p["avg_ms"] * 1e-3) / 1e12}, p)


def host_pmu(ctx, expanded):
    """The exact replay's host counters (ulg_get_info exact_*: perf_event_open
    on the replay thread, user space): cycles, instructions and the kernel's
    generic cache-miss event per expansion -- the replay's floor as numbers.
    None where the host does not grant the counters."""
    try:
        cyc, ins, mis = (ctx.info(k) for k in ("exact_cycles", "exact_instructions", "exact_cache_misses"))
    except Exception:  # noqa: BLE001 -- an older library
        return None
    e = max(int(expanded), 1)
    out = {"event": "PERF_COUNT_HW_CPU_CYCLES / _INSTRUCTIONS / _CACHE_MISSES, user space, replay thread"}
    out["cycles_per_expansion"] = cyc / e if cyc >= 0 else None
    out["instructions_per_expansion"] = ins / e if ins >= 0 else None
    out["ipc"] = ins / cyc if cyc > 0 and ins >= 0 else None
    out["cache_misses_per_expansion"] = mis / e if mis >= 0 else None
    return out if any(out[k] is not None for k in ("cycles_per_expansion", "cache_misses_per_expansion")) else None


# round 6: FETCH/WRITE passes of the sweep kernel HEAD launches (scripts/pmc_search.sh)
PMC_SEARCH = os.path.join(os.path.dirname(PROFILES), "r6", "pmc_search_traffic.json")


def search_roofline(cfg, n, pull, reps):
    """Roofline of the GPU order-graph sweep (layer_pull_w32_kernel at C3,
    search_gpu.hip, one launch per layer) on a full skeleton: a layer-L node reads L predecessors' g
    (4 B) and best-score costs (4 B, the 32-bit lattice) and writes its g
    (4 B) and leaf (1 B), so one sweep's algorithmic bytes are
    sum_L C(n, L) (8 L + 5).  The achieved rate divides them by the sweep's
    summed kernel time (HIP events on the launch stream); traffic is the
    PMC-measured bytes of one sweep."""
    cnt, sweep_ms = pull["count"], pull["total_ms"] / reps
    algo = sum(math.comb(n, L) * (8 * L + 5) for L in range(1, n + 1))
    achieved = algo / (sweep_ms * 1e-3) / 1e9
    traffic, src, kern = None, None, pull.get("kernel", "layer_pull_w32_kernel")
    try:
        t = json.load(open(PMC_SEARCH))
        if t.get("config_id") == cfg["id"] and t.get("n") == n:
            traffic, src = t["traffic_bytes_per_sweep"], os.path.relpath(PMC_SEARCH, ROOT)
            kern = t.get("kernel", kern)
    except (OSError, ValueError):
        pass
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per sweep",
            "traffic_source": src, "kernel": kern, "launches_per_sweep": cnt // reps,
            "sweep_kernel_ms": sweep_ms, "algorithmic_bytes_per_sweep": algo,
            "bytes_per_node": "8 L + 5 (L predecessors x (4 B g + 4 B best-score cost) + 4 B g + 1 B leaf written)"}


def search_metrics(ctx, cfg, variables, cands, rank, ws, reps=3, edges=None, skel_note="full skeleton",
                   loaded=False, lists=None):
    """Order-graph search side: GPU best-score tables + pattern database +
    the GPU layer-synchronous search at the bench config (time to the optimal
    order cost; it settles every lattice node, so its rate is lattice nodes/s,
    not A* expansions), then the exact-order A* (the reference's pop order,
    bit-exact DAG; true A* expansions/s) and a bounded sample of the CPU
    oracle's A* at the same config (rank 0, N=1 only; exact_astar_legs).
    loaded: the lists are already in the search state (ulg_search_load_scores
    after the exchange); lists: the same lists on the host (offsets, sets,
    scores) for the CPU leg."""
    import time as _t
    n, k = cfg["n"], cfg["k"]
    full = [(1 << n) - 1] * n
    skel = full if edges is None else edges
    out = {}
    tables_ms = tables_again_ms = None
    if not loaded:
        stored, _ = ctx.score(list(range(n)), full if edges is None else ulg.candidates_from_edges(edges, n), k)
        if lists is None and rank == 0 and ws == 1:
            lists = ctx.fetch(stored)
        t0 = _t.perf_counter()
        ctx.search_from_scores()
        tables_ms = 1e3 * (_t.perf_counter() - t0)
        t1 = _t.perf_counter()
        ctx.search_from_scores()  # again, with the tables already allocated (3.4 GB at C3)
        tables_again_ms = 1e3 * (_t.perf_counter() - t1)
    t1 = _t.perf_counter()
    ctx.pdb_build(2)
    t2 = _t.perf_counter()
    # HIP events around every layer_pull_kernel launch of the sweeps and the
    # one-time sweep-table build (search_sweep_w: the first call lays the
    # successor costs out in the sweep's order; later calls reuse it)
    ctx.profile(True)
    ctx.profile_select(["search_layer_pull", "search_sweep_w"])
    ctx.profile_reset()
    times = []
    for _ in range(reps):
        ts = _t.perf_counter()
        g = ctx.astar(edges=skel, mode=1, net_text=False)
        times.append(_t.perf_counter() - ts)
    pull = ctx.profile_get("search_layer_pull")
    wb = ctx.profile_get("search_sweep_w")
    ctx.profile(False)
    first, best = times[0], min(times[1:]) if reps > 1 else times[0]
    out["gpu_search"] = {"config": f"{cfg['id'].upper()} lists (n={n}, k={k}), {skel_note}, static PDB(2)",
                         "lattice_nodes": g["expanded"], "time_to_optimal_cost_ms": 1e3 * first,
                         "lattice_nodes_per_s": g["expanded"] / first, "goal_cost": g["cost"],
                         "repeat_call_ms": 1e3 * best,
                         "sweep_table_ms": wb["total_ms"] if wb else None,
                         "tables_ms": tables_ms, "tables_rebuild_ms": tables_again_ms,
                         "pdb_ms": 1e3 * (t2 - t1),
                         "note": "layer-synchronous pull over the whole order lattice (every node settled, "
                                 "so nodes/s is not an A* expansion rate); time_to_optimal_cost_ms = the first "
                                 "call after the tables (incl. the sweep-table build), repeat_call_ms = best of "
                                 "%d later calls" % (reps - 1)}
    if edges is None and pull is not None:
        out["gpu_search"]["roofline"] = search_roofline(cfg, n, pull, reps)
    if rank == 0 and ws == 1 and lists is not None:
        out.update(exact_astar_legs(ctx, cfg, skel, lists))
    return out

GOLDEN = os.path.join(ROOT, "tests", "golden")


def exact_astar_legs(ctx, cfg, skel, lists, oracle_budget_s=15.0):
    """The headline's A* half at the bench config: the exact-order A*
    (run_astar_on_one_scc, astar_main.cpp:266-459: the reference's heap and
    pop order replayed on the host over the GPU-built O(1) tables) from the
    root push to the goal pop, reported as expansions/s, with its netFile
    checked against the oracle command lines' (tests/golden/<config>_oracle.json
    when the config has one); then the CPU oracle's A* (sorted-list scans,
    reference heap, one thread like the reference) on the same lists for a
    bounded wall-clock budget (its -r watchdog), reported as expansions/s over
    that sample with the open-list size it reached."""
    import time as _t
    n = cfg["n"]
    out = {}
    ts = _t.perf_counter()
    e = ctx.astar(edges=skel, mode=0, net_text=True)
    dt = _t.perf_counter() - ts
    fx = os.path.join(GOLDEN, f"{cfg['id']}_oracle.json")
    same = None
    if os.path.exists(fx):
        ref = json.load(open(fx))
        same = (e["net_text"] == ref["net_file"] and e["expanded"] == ref["expanded"]
                and np.float32(e["cost"]).tobytes() == np.float32(ref["goal_cost"]).tobytes())
    out["exact"] = {"config": f"{cfg['id'].upper()} (n={n}, N={cfg['N']}, k={cfg['k']}), "
                              + ("full skeleton" if skel == [(1 << n) - 1] * n else "skeleton"),
                    "expansions": e["expanded"], "ms": 1e3 * dt, "expansions_per_s": e["expanded"] / dt,
                    "ns_per_expansion": 1e9 * dt / max(e["expanded"], 1),
                    "goal_cost": e["cost"],
                    "host_pmu": host_pmu(ctx, e["expanded"]),
                    "same_netfile_cost_expansions_as_oracle_fixture": same,
                    "oracle_fixture": os.path.relpath(fx, ROOT) if os.path.exists(fx) else None,
                    "note": "reference pop order replayed on the host over GPU-built O(1) tables; the time "
                            "includes the successor-cost rows' build and copy (first call)"}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    offs, sets, scores = lists
    costs = ctx.quantize(scores)
    srch = oracle.Search(n, offs, sets, costs)
    ts = _t.perf_counter()
    srch.pdb_build(2)
    pdb_s = _t.perf_counter() - ts
    ts = _t.perf_counter()
    r = srch.astar(edges=skel, time_limit_s=oracle_budget_s)
    dt = _t.perf_counter() - ts
    full_run = None
    if os.path.exists(fx):
        ref = json.load(open(fx))
        full_run = (f"the oracle's full run of this config (make_c3_fixture.py, build container's CPU): "
                    f"{ref['expanded']} expansions in {ref['oracle_astar_seconds']:.0f} s = "
                    f"{ref['expanded'] / ref['oracle_astar_seconds']:.0f} expansions/s")
    out["cpu_baseline"] = {
        "value": r["expanded"] / dt, "unit": "A* expansions/s", "cores": 1, "kind": "port", "cpu": cpu_model(),
        "sample": f"CPU oracle A* (sorted-list getScore scans, hashed generatedNodes, reference heap) on the "
                  f"{cfg['id'].upper()} lists, stopped by its -r watchdog after {dt:.1f} s: {r['expanded']} "
                  f"expansions, open list {r['open_list']} nodes "
                  f"({'goal reached' if not r['out_of_time'] else 'goal not reached'}); PDB build "
                  f"{pdb_s:.2f} s outside the timed region",
        "full_run": full_run,
        "expansions_reached_fraction_of_exact": r["expanded"] / max(e["expanded"], 1)}
    return out


def c4_leg(device, budget_s=1.0):
    """BASELINE config C4 beside the headline (rank 0, N = 1): n=30, N=100k,
    the MMPC skeleton built on the GPU from the same data (alpha 0.01), 2-hop
    candidate sets (score_main.cpp:146-153) and the reference's default
    parent limit -p = n - 1 (score_main.cpp:296-298), so layers 9..18 run the
    wide kernels.  One step = one complete synchronised scoring call over all
    30 variables (every call decides every parent set; the wide layers sync
    for their queue lengths, so steps are not overlapped); steps are repeated
    for about budget_s after two warm-up calls.  The three variables of
    tests/golden/c45_oracle.json (the oracle's lists, up to 52 min each) are
    checked by count and SHA-256 after the timed calls."""
    cfg = dict(CONFIGS["c4"], id="c4")
    n, N, k = cfg["n"], cfg["N"], cfg["k"]
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx = ulg.Context(device)
    try:
        t0 = time.perf_counter()
        ctx.load(X, cfg["lam"])
        rows = ctx.mmpc(cfg["alpha"])
        prep_ms = 1e3 * (time.perf_counter() - t0)
        cands = ulg.candidates_from_edges(rows, n)
        variables = list(range(n))
        for _ in range(2):
            ctx.score(variables, cands, k)
        ts = []
        scored = stored = 0
        tb = time.perf_counter()
        while not ts or (time.perf_counter() - tb < budget_s and len(ts) < 200):
            a = time.perf_counter()
            stored, scored = ctx.score(variables, cands, k)
            ts.append(time.perf_counter() - a)
        offs, sets, _ = ctx.fetch(stored)
        chk = lists_vs_fixture(cfg, variables, offs, sets)
        if chk is not None and chk[1]:
            raise RuntimeError(f"bench.py: C4 lists differ from tests/golden/c45_oracle.json for variables {chk[1]}")
        msz = [bin(c & ~(1 << v)).count("1") for v, c in enumerate(cands)]
        return {"workload": "C4 cBIC scoring: n=30, N=100000, MMPC skeleton (ulg_mmpc alpha 0.01, "
                            f"{sum(bin(r).count('1') for r in rows) // 2} edges), 2-hop candidate sets "
                            f"(largest {max(msz)}), -p 29 (the reference's default n - 1), all 30 variables",
                "steps": len(ts), "ms_per_step": 1e3 * float(np.mean(ts)),
                "ms_per_step_median": 1e3 * float(np.median(ts)), "ms_per_step_min": 1e3 * float(np.min(ts)),
                "value": scored / float(np.mean(ts)), "unit": "parent-set scores/s",
                "parent_sets_per_step": scored, "stored_per_step": stored,
                "load_and_mmpc_ms": prep_ms,
                "lists_equal_oracle": (chk is not None and not chk[1]),
                "oracle_variables_checked": chk[0] if chk else [],
                "note": "synchronised calls timed on the host clock (data resident in HBM); the oracle check "
                        "covers the fixture's variables (counts + SHA-256 of the sorted masks)"}
    finally:
        ctx.close()


def cpu_quota():
    """The cgroup CPU bandwidth limit (cpu.max), which can be far below nproc:
    threads beyond it time-share."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """--gpus N without a launcher: one worker process per GPU, started before
    this process touches the GPU; returns the worst exit status."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def lists_digest(offsets, sets, scores):
    """SHA-256 over (offsets, sets, score bits) of the gathered lists."""
    h = hashlib.sha256()
    h.update(np.asarray(offsets, dtype=np.int64).tobytes())
    h.update(np.asarray(sets).view(np.uint64).tobytes())
    h.update(np.asarray(scores, dtype=np.float32).tobytes())
    return h.hexdigest()


def lists_vs_fixture(cfg, variables, offs, sets):
    """Compare one context's stored lists with the oracle command lines'
    per-variable counts and SHA-256 digests of the sorted masks
    (tests/golden/<config>_oracle.json for C2/C3; c45_oracle.json's sampled
    variables for C4).  Returns (checked variables, mismatching variables),
    or None when no fixture covers this config."""
    fx = os.path.join(GOLDEN, f"{cfg['id']}_oracle.json")
    per = {}
    if os.path.exists(fx):
        ref = json.load(open(fx))
        for v in range(cfg["n"]):
            per[v] = (ref["stored_per_variable"][v], ref["sets_sha256_per_variable"][v])
    elif cfg["id"] == "c4" and os.path.exists(os.path.join(GOLDEN, "c45_oracle.json")):
        ref = json.load(open(os.path.join(GOLDEN, "c45_oracle.json")))["c4"]
        for vs, r in ref["per_variable"].items():
            per[int(vs)] = (r["stored"], r["sets_sha256"])
    else:
        return None
    checked, bad = [], []
    for i, v in enumerate(variables):
        if v not in per:
            continue
        s = np.sort(np.asarray(sets[offs[i]:offs[i + 1]]).astype(np.uint64))
        checked.append(v)
        if len(s) != per[v][0] or hashlib.sha256(s.tobytes()).hexdigest() != per[v][1]:
            bad.append(v)
    return checked, bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default 1, or WORLD_SIZE under a launcher")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="shard", choices=["shard", "weak"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-search", action="store_true")
    ap.add_argument("--no-c4", action="store_true", help="skip the extra C4 object (N=1 only)")
    ap.add_argument("--score-variant", type=int, default=None, help="A/B knob (ulg_set_option score_variant)")
    ap.add_argument("--option", action="append", default=[], help="A/B knob name=value (ulg_set_option)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + --device: rehearse the N>1 code path with several ranks on one GPU")
    ap.add_argument("--device", type=int, default=None, help="GPU for every rank (default LOCAL_RANK)")
    ap.add_argument("--slots", type=int, default=None,
                    help="scoring steps in flight per rank: contexts whose calls are queued with "
                         "ulg_cbic_score_async and collected slots - 1 steps later (every step complete); "
                         "with more than one, each context scores on one stream (score_streams 1) unless "
                         "--option score_streams=... says otherwise (default 3 when every layer is unrolled, "
                         "k <= 8; 1 for the wide layers of C1/C4, whose calls synchronise anyway)")
    args = ap.parse_args()
    if args.slots is None:
        args.slots = 3 if CONFIGS[args.config]["k"] <= 8 else 1
    if args.slots > 1 and not any(o.startswith("score_streams=") for o in args.option):
        # independent steps in flight replace the stream groups as the source of
        # concurrency: one chain per context, S chains at once (C3: 1.18 ms per
        # step with 1 slot x 3 groups, 0.67 ms with 3 slots x 1 stream;
        # profiles/r3/slots/)
        args.option.append("score_streams=1")
    if args.slots > 1 and not any(o.startswith("walk_k6=") for o in args.option):
        # throughput with steps in flight: 8 sets per lane share one walk of
        # the layer-6 union tree (10.17e9 against 9.80e9 sets/s with 4; the
        # single-call context below keeps the library default, 4)
        args.option.append("walk_k6=8")

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    ws, rank, local = dist_env()
    if args.gpus is not None and args.gpus != ws:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
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
        ws = dist.get_world_size()
    else:
        torch.cuda.set_device(local)

    seed = 9200 + (rank if args.mode == "weak" else 0)
    X, _ = synth.gaussian_sem(n, N, seed)
    ctx = ulg.Context(local)
    if args.score_variant is not None:
        ctx.set_option("score_variant", args.score_variant)
    for kv in args.option:
        k_, v_ = kv.split("=", 1)
        ctx.set_option(k_, int(v_))
    ctx.load(X, lam)
    cands_all = [(1 << n) - 1] * n
    skel_note = "full n x n skeleton"
    rows = None
    if cfg.get("skeleton") == "mmpc":
        rows = ctx.mmpc(cfg["alpha"])
        cands_all = ulg.candidates_from_edges(rows, n)
        skel_note = (f"MMPC skeleton (ulg_mmpc, alpha {cfg['alpha']}: {sum(bin(r).count('1') for r in rows) // 2} "
                     f"edges), 2-hop candidate sets")
    ex = None
    if args.mode == "shard":
        parts = shard.assign(n, ws, cands_all, k)
        variables = parts[rank]
        if ws > 1:
            ex = shard.ListExchange(n, parts, cands_all, k, rank, device="cuda", comm_device=cdev)
    else:
        variables = list(range(n))
    cands = [cands_all[v] for v in variables]
    units_rank = sum(shard.var_weight(n, v, cands_all[v], k) for v in variables)
    msz = [bin(cands_all[v] & ~(1 << v)).count("1") for v in range(n)]

    def step():
        stored, scored = ctx.score(variables, cands, k)
        if ex is not None:
            ex.fill(ctx, stored)
            ex.allgather()  # the one collective of the data path
        return scored

    # --slots S > 1: S contexts on this GPU (same data), step i on context
    # i % S; its scoring call is queued without waiting and collected (then
    # its lists exchanged) S - 1 steps later, so the latency-bound parts of
    # one step's launch chain overlap the next steps' work.  Collectives stay
    # in step order on one thread.
    slots = max(1, args.slots)
    sctx, sex = [ctx], [ex]
    for _ in range(slots - 1):
        c2 = ulg.Context(local)
        for kv in args.option:
            k_, v_ = kv.split("=", 1)
            c2.set_option(k_, int(v_))
        if args.score_variant is not None:
            c2.set_option("score_variant", args.score_variant)
        c2.load(X, lam)
        sctx.append(c2)
        sex.append(shard.ListExchange(n, parts, cands_all, k, rank, device="cuda", comm_device=cdev)
                   if ex is not None else None)

    def run_steps(nsteps):
        """nsteps complete steps; returns the sets scored and the steps run on context 0."""
        if slots == 1:
            return sum(step() for _ in range(nsteps)), nsteps
        total, pend, on0 = 0, [], 0

        def complete(s):
            stored, scored = sctx[s].score_finish()
            if sex[s] is not None:
                sex[s].fill(sctx[s], stored)
                sex[s].allgather()
            return scored
        for i in range(nsteps):
            s = i % slots
            on0 += s == 0
            sctx[s].score_async(variables, cands, k)
            pend.append(s)
            if len(pend) == slots:
                total += complete(pend.pop(0))
        while pend:
            total += complete(pend.pop(0))
        return total, on0

    run_steps(max(args.warmup, slots))
    # HIP events in the timed region only around the roofline unit's kernels
    # (two host-side event records per timed kernel would otherwise show up in
    # a ~1.5 ms step of ~35 launches); the full per-kernel breakdown comes from
    # one extra profiled step after it
    kk = min(k, max(msz[v] for v in variables)) if variables else k
    ctx.profile(True)
    ctx.profile_select([r.format(k=kk) for r in ROOF_KERNELS])
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scored_total, steps_ctx0 = run_steps(args.steps)
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
    per_launch = sum(math.comb(msz[v] - (1 if (v != 0 and cands_all[v] & 1) else 0), kk) for v in variables)
    if ex is not None and slots > 1:
        # every slot's last exchange holds the whole job's lists: all equal
        ds = set()
        for e in sex:
            o_, st_, sc_ = e.assemble()
            ds.add(lists_digest(o_, st_.cpu().numpy(), sc_.cpu().numpy()))
        if len(ds) != 1:
            raise RuntimeError(f"bench.py: the {slots} slots exchanged different lists")
    # The lists the timed steps left on EVERY slot context (the last step each
    # context ran, graph replay included) against the oracle command lines'
    # per-variable digests; a mismatch fails the bench.
    slot_check = None
    if ex is None:
        checked_all, bad_all = set(), {}
        for si, c in enumerate(sctx):
            st_, _ = c.score_finish()
            o_, s_, _ = c.fetch(st_)
            r = lists_vs_fixture(cfg, variables, o_, s_)
            if r is None:
                break
            checked_all.update(r[0])
            if r[1]:
                bad_all[si] = r[1]
        else:
            if bad_all:
                raise RuntimeError(f"bench.py: slot contexts' lists differ from the oracle fixture: {bad_all}")
            slot_check = {"slots_lists_equal_oracle": True, "contexts": slots,
                          "variables_checked": len(checked_all),
                          "fixture": f"tests/golden/{cfg['id']}_oracle.json"}
    # Non-overlapped measurement (after the timed region): context 0 alone,
    # one call at a time on one stream, HIP events on the roofline kernels'
    # launch stream -- their durations are not stretched by concurrent steps,
    # so the dominant kernel's time per call is below the call's own time.
    ctx.set_option("score_streams", 1)
    ctx.profile(True)
    ctx.profile_select([r.format(k=kk) for r in ROOF_KERNELS])
    ctx.profile_reset()
    solo_calls = 5
    ts_solo = []
    for _ in range(solo_calls):
        torch.cuda.synchronize()
        a = time.perf_counter()
        ctx.score(variables, cands, k)
        ts_solo.append(time.perf_counter() - a)
    step_bytes = sum(math.comb(msz[v], L) * 4 * (L + 1) for v in variables for L in range(0, k + 1))
    roof, _ = roofline(ctx, dict(cfg, k=kk, msz=[msz[v] for v in variables]), per_launch, solo_calls)
    ctx.profile(False)
    if roof is not None:
        roof["note"] = ("one call at a time on one stream (context 0 after the timed region, %d calls): the "
                        "dominant pair's launches do not overlap other work" % solo_calls)
        roof["solo_call_ms"] = 1e3 * float(np.median(ts_solo))
    # single_call_ms: what one drop-in call (bin/score, ulg_cbic_score) takes
    # with the library's default options on a fresh context, synchronised
    single = ulg.Context(local)
    single.load(X, lam)
    for _ in range(2):
        single.score(variables, cands, k)
    ts_single = []
    for _ in range(10):
        torch.cuda.synchronize()
        a = time.perf_counter()
        single.score(variables, cands, k)
        ts_single.append(time.perf_counter() - a)
    single.close()
    single_call_ms = 1e3 * float(np.median(ts_single))
    if roof is not None:
        # the same compulsory bytes (4 (L + 1) per set) over the whole step:
        # every layer of every variable of this rank, per ms_per_step
        roof["step_level"] = {"algorithmic_bytes_per_step": step_bytes,
                              "achieved_gbs": step_bytes / (elapsed / args.steps) / 1e9,
                              "frac": step_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS,
                              "note": "all of this rank's sets per timed step (the per-launch figure above is "
                                      "the dominant kernel's; concurrent steps stretch each launch)"}
    ctx.profile(True)
    ctx.profile_select(None)
    ctx.profile_reset()
    step()
    kernels = ctx.profile_dump()
    ctx.profile(False)

    # split of the sharded step, measured after the timed region: scoring
    # alone vs scoring + exchange (synchronised, so not part of `value`)
    split = None
    if ex is not None:
        ts_score, ts_ex = [], []
        for _ in range(max(3, min(args.steps, 10))):
            if dist:
                dist.barrier()
            torch.cuda.synchronize()
            a = time.perf_counter()
            stored, _ = ctx.score(variables, cands, k)
            ex.fill(ctx, stored)
            torch.cuda.synchronize()
            b = time.perf_counter()
            ex.allgather()
            torch.cuda.synchronize()
            c = time.perf_counter()
            ts_score.append(b - a)
            ts_ex.append(c - b)
        stored_bytes = sum(ex.counts) * (ex.w + 4)
        split = {"score_ms": 1e3 * float(np.median(ts_score)), "exchange_ms": 1e3 * float(np.median(ts_ex)),
                 "exchange_bytes_per_rank": ex.block, "exchange_bytes_total": ex.block * ws,
                 "block_capacity_sets": ex.cap, "a_priori_capacity_sets": ex.bound,
                 "stored_sets_total": sum(ex.counts), "stored_bytes_total": stored_bytes,
                 "exchange_over_stored_bytes": ex.block * ws / max(stored_bytes, 1), "regathers": ex.regathers,
                 "note": "medians of synchronised steps after the timed region (rank-local clocks); blocks "
                         "sized by the learned capacity (the largest rank's stored count + 2% + 256 sets; the "
                         "first exchange used the a-priori bound)"}

    search = None
    if args.mode == "shard" and not args.no_search:
        search = sharded_search(ctx, cfg, ex, variables, cands, rows, skel_note, rank, ws, dist, cdev, torch)
    elif args.mode == "weak" and not args.no_search:
        search = search_metrics(ctx, cfg, variables, cands, rank, ws, edges=rows, skel_note=skel_note)

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
                                   f"lambda={lam}, {skel_note}, "
                                   + (f"all {n} variables per GPU" if args.mode == "weak" else
                                      f"{n} variables balanced over {ws} GPU(s), one all-gather of the lists"),
                       "config_id": args.config, "mode": args.mode,
                       "parallelism": f"variable shard x{ws}" if args.mode == "shard" else f"replicas x{ws}",
                       "steps_in_flight": slots,
                       "parent_sets_per_step_per_rank": units_rank},
            "roofline": roof,
            "kernel_ms_one_step": {kk2: round(vv["total_ms"], 4) for kk2, vv in kernels.items()},
        }
        res["single_call_ms"] = single_call_ms
        res["single_call_note"] = ("one synchronised ulg_cbic_score call at a time with the library's default "
                                   "options (what bin/score makes), median of 10 on a fresh context")
        if slot_check is not None:
            res["slot_check"] = slot_check
        if split is not None:
            res["shard_step"] = split
        if search is not None:
            res["astar"] = search
        if ws == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg, X)
        if ws == 1 and args.config != "c4" and not args.no_c4:
            res["c4"] = c4_leg(local)
        print(json.dumps(res), flush=True)
    for c2 in sctx[1:]:
        c2.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def sharded_search(ctx, cfg, ex, variables, cands, rows, skel_note, rank, ws, dist, cdev, torch):
    """After the exchange: every rank holds every variable's list, builds its
    own best-score tables and pattern database and runs the GPU order-graph
    search (replicas).  Ranks must agree on the lists (digest) and
    the goal cost."""
    n = cfg["n"]
    host_lists = None
    if ex is not None:
        stored, _ = ctx.score(variables, cands, cfg["k"])
        ex.fill(ctx, stored)
        ex.allgather()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        offsets, sets_t, scores_t = ex.assemble(device="cuda")
        t1 = time.perf_counter()

        def load():
            ctx.search_load_scores(offsets, sets_t.data_ptr(), scores_t.data_ptr(), device_ptrs=True)
        digest = lists_digest(offsets, sets_t.cpu().numpy(), scores_t.cpu().numpy())
    else:
        stored, _ = ctx.score(variables, cands, cfg["k"])
        offs, sets, scores = ctx.fetch(stored)
        host_lists = (offs, sets, scores)
        t0 = t1 = time.perf_counter()

        def load():
            ctx.search_load_scores(offs, sets, scores, device_ptrs=False)
        digest = lists_digest(offs, sets, scores)
    ta = time.perf_counter()
    load()
    tb = time.perf_counter()
    load()  # again, with the tables already allocated (3.4 GB at C3)
    tc = time.perf_counter()
    out = search_metrics(ctx, cfg, variables, cands, rank, ws, edges=rows, skel_note=skel_note, loaded=True,
                         lists=host_lists)
    out["gpu_search"].update(assemble_ms=1e3 * (t1 - t0), tables_ms=1e3 * (tb - ta), tables_rebuild_ms=1e3 * (tc - tb))
    out["lists_sha256"] = digest
    if dist and ws > 1 and rows is None:
        # SURVEY 8e's n >= 31 path at this n: tables and sweep slices sharded
        # by variable, one MIN all-reduce of each layer's (cost, leaf) keys
        own = shard.table_owners(n, ws)[rank]
        dist.barrier()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        res = shard.sharded_sweep(ctx, n, own, device="cuda", comm_device=cdev)
        tb = time.perf_counter()
        out["table_sharded_sweep"] = {
            "ms": 1e3 * (tb - ta), "goal_cost": res["cost"],
            "same_as_replica": bool(np.float32(res["cost"]).tobytes()
                                    == np.float32(out["gpu_search"]["goal_cost"]).tobytes()),
            "own_variables": bin(own).count("1"),
            "note": "this rank's tables + sweep slices for its own variables, then n layers of "
                    "(local keys, one MIN all-reduce, commit); rank-local clock"}
    if dist:
        # every rank must hold the same lists and find the same goal cost
        h = torch.tensor([int(digest[:15], 16), int(np.float32(out["gpu_search"]["goal_cost"]).view(np.int32))],
                         dtype=torch.int64, device=cdev)
        lo, hi = h.clone(), h.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        out["ranks_agree"] = bool(torch.equal(lo, hi))
    return out


if __name__ == "__main__":
    main()
