"""Time the search side at a BASELINE config on the GPU (diagnostic)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import numpy as np
import synth, ulg

n, N, k = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
exact = len(sys.argv) > 4 and sys.argv[4] == "exact"
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
full = [(1 << n) - 1] * n
ctx.profile(True)
out = {}
t = time.perf_counter(); st, sc = ctx.score(list(range(n)), full, k); out["score_s"] = time.perf_counter() - t
out["stored"] = st
t = time.perf_counter(); ctx.search_from_scores(); out["tables_s"] = time.perf_counter() - t
t = time.perf_counter(); ctx.pdb_build(2); out["pdb_s"] = time.perf_counter() - t
for rep in range(2):
    t = time.perf_counter(); g = ctx.astar(edges=full, mode=1, net_text=False); out[f"gpu_search_s_{rep}"] = time.perf_counter() - t
out["gpu_cost"] = g["cost"]; out["gpu_expanded"] = g["expanded"]
if exact:
    t = time.perf_counter(); e = ctx.astar(edges=full, mode=0, net_text=False); out["exact_s"] = time.perf_counter() - t
    out["exact_cost"] = e["cost"]; out["exact_expanded"] = e["expanded"]
    out["same_dag"] = [int(x) for x in e["vpar"]] == [int(x) for x in g["vpar"]]
out["kernels"] = ctx.profile_dump()
print(json.dumps(out))
