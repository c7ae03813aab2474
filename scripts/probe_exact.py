"""Times the exact-order A* (host replay over GPU tables) at C2 and C3, with
the replay thread's host counters per expansion (ulg_get_info exact_*), and
checks C3's goal cost and expansion count against tests/golden/c3_oracle.json.
ULG_EXACT_PF selects the heap layout / prefetch mode (search_host.cpp):
    python scripts/probe_exact.py [c2] [c3]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402

ctx = ulg.Context(0)
CFG = {"c2": (20, 10000, 4), "c3": (25, 10000, 6)}
for name in (sys.argv[1:] or ["c2", "c3"]):
    n, N, k = CFG[name]
    X, _ = synth.gaussian_sem(n, N, 9200)
    full = [(1 << n) - 1] * n
    ctx.load(X, 2.0)
    ctx.score(list(range(n)), full, k)
    ctx.search_from_scores()
    t = time.perf_counter()
    r = ctx.astar(edges=full, mode=0, net_text=(name == "c3"))
    dt = time.perf_counter() - t
    e = max(r["expanded"], 1)
    pmu = {kk: ctx.info("exact_" + kk) for kk in ("cycles", "instructions", "cache_misses")}
    out = {"case": name, "pf": os.environ.get("ULG_EXACT_PF", "6"), "expanded": r["expanded"], "seconds": dt,
           "expansions_per_s": r["expanded"] / dt, "cost": r["cost"],
           "ns_per_expansion": 1e9 * dt / e,
           "cycles_per_expansion": pmu["cycles"] / e if pmu["cycles"] >= 0 else None,
           "cache_misses_per_expansion": pmu["cache_misses"] / e if pmu["cache_misses"] >= 0 else None}
    if name == "c3":
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", "c3_oracle.json")))
        out["oracle_expanded"] = ref.get("expanded")
        out["equal_to_oracle"] = (r["expanded"] == ref["expanded"] and r["cost"] == ref["goal_cost"]
                                  and r["net_text"] == ref["net_file"])
    print(json.dumps(out), flush=True)
