"""Debug probe (GPU box): ulg_triplet_astar vs the oracle on one sparse case,
plus pattern-database parity over the triples' clusters of that case."""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "urlearning-cpp_amd")]
import oracle as o  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402

seed, n, extra, k = 9405, 16, 0.05, 3
X, W = synth.gaussian_sem(n, 3000, seed)
rows = synth.true_skeleton_edges(W, extra, seed)
rows = [r & ~(1 << i) for i, r in enumerate(rows)]
cands = ulg.candidates_from_edges(rows, n)
ds = o.Dataset(X)
offs, sets, scores = ds.score_all(2.0, cands, k, threads=8)
costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
ctx = ulg.Context(0)
ctx.search_load(offs, sets, costs)
srch = o.Search(n, offs, sets, costs)
res = ctx.triplet(edges=rows)
ref = o.triplet(srch, edges=rows)
print("gpu stats", res["runs"], res["distinct"], res["expanded"])
print("ora stats", ref["runs"], ref["distinct"], ref["expanded"])
print("mec diff at", np.argwhere(res["mec"] != ref["mec"]).tolist())
clusters = [r | (1 << v) for v, r in enumerate(rows)]
seen = set()
bad = 0
for i, j, kk in itertools.combinations(range(n), 3):
    big = clusters[i] | clusters[j] | clusters[kk]
    if big in seen:
        continue
    seen.add(big)
    srch.pdb_build(2, 0, big)
    ctx.pdb_build(2, 0, big)
    bits = [b for b in range(n) if (big >> b) & 1]
    Ss = [sum(1 << bits[t] for t in range(len(bits)) if (m >> t) & 1) for m in range(1 << len(bits))]
    h, comp = ctx.pdb_h(Ss)
    for S, hv, cv in zip(Ss, h, comp):
        eh, ec = srch.pdb_h(S)
        if np.float32(hv).tobytes() != np.float32(eh).tobytes() or int(cv) != ec:
            bad += 1
            if bad < 10:
                print("pdb mismatch cluster", hex(big), "S", hex(S), hv, eh, cv, ec)
    # the lattice lookups the search makes inside the cluster
    qv, qS = [], []
    for S in Ss[:512]:
        for v in bits:
            qv.append(v)
            qS.append(S | (1 << v))
    gc, gp = ctx.bestscore(qv, qS)
    for v, S, c, p in zip(qv, qS, gc, gp):
        ec, ep = srch.bestscore(v, S)
        if np.float32(c).tobytes() != np.float32(ec).tobytes() or int(p) != ep:
            bad += 1
            if bad < 20:
                print("bs mismatch", v, hex(S), c, ec, int(p), ep)
print("clusters", len(seen), "mismatches", bad)
