"""GPU search at C4 (n=30, N=100k, MMPC skeleton, 2-hop candidates, k=8):
per-kernel split of the layer-synchronous search (diagnostic)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth, ulg
n, N, k = 30, 100000, 8
X, _ = synth.gaussian_sem(n, N, 9200)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
rows = ctx.mmpc(0.01)
cands = ulg.candidates_from_edges(rows, n)
ctx.score(list(range(n)), cands, k)
ctx.search_from_scores()
ctx.pdb_build(2)
g = ctx.astar(edges=rows, mode=1, net_text=False)
ctx.profile(True)
ctx.profile_reset()
t = time.perf_counter()
g = ctx.astar(edges=rows, mode=1, net_text=False)
dt = time.perf_counter() - t
prof = ctx.profile_dump()
print(json.dumps({"ms": 1e3 * dt, "expanded": g["expanded"], "cost": g["cost"],
                  "edges": sum(bin(r).count("1") for r in rows) // 2,
                  "kernels": {kk: (v["count"], round(v["total_ms"], 3)) for kk, v in
                              sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])[:12]}}))
