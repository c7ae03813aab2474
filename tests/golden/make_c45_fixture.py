#!/usr/bin/env python3
"""Generate tests/golden/c45_oracle.json: the CPU oracle's stored parent-set
lists for a few variables of BASELINE configs C4 and C5, on the seeded
synthetic data bench.py and the tests use.

  C4: n=30, N=100k, synth.gaussian_sem(30, 100000, 9200), MMPC skeleton
      (oracle ora_mmpc, alpha 0.01; the GPU's ulg_mmpc equals it), 2-hop
      candidate sets (score_main.cpp:146-153), the reference's default
      parent limit -p = n - 1 (score_main.cpp:296-298), lambda 2.
  C5: n=32, N=50k, synth.gaussian_sem(32, 50000, 9200), full skeleton,
      k = 6 (the k-capped variant), lambda 2.

Every variable here is scored by ora_score_variable (the faithful
restatement: per-set OLS over all N rows, BIC_OLS.cpp:174-389, in Gosper
order, score_calculator.cpp:54-135).  Per variable the fixture keeps the
stored-set count, a SHA-256 of the sorted uint64 masks, the float64 sum of
the float32 scores, and every 512th stored (set, score) pair in sorted-set
order so the test can hold each sampled score to 1e-6 relative.

This runs in this container only (it needs oracle/build/; the full set is
about five hours of CPU):  python tests/golden/make_c45_fixture.py [procs]
Variables already in the committed fixture are kept (same data, same
skeleton), only the missing ones are run, and the file is rewritten after
every finished variable so a partial run keeps what it has.
"""
import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "urlearning-cpp_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import synth  # noqa: E402

LAM, SEED, STRIDE = 2.0, 9200, 512
CONFIGS = {
    # C4: every variable (round 6; cost grows ~2.2x per candidate, the
    # m = 18 variable 9 takes ~52 min, m = 17 variable 23 ~20 min).
    "c4": dict(n=30, N=100000, k=29, skeleton="mmpc", alpha=0.01, variables=list(range(30))),
    # C5: 8 variables spread over the order (~41 min each).
    "c5": dict(n=32, N=50000, k=6, skeleton="full", variables=[0, 5, 9, 13, 17, 21, 25, 31]),
}


def candidates(cfg, ds):
    import ulg
    n = cfg["n"]
    if cfg["skeleton"] == "full":
        return [(1 << n) - 1] * n, None
    rows = ds.mmpc(cfg["alpha"])
    return ulg.candidates_from_edges(rows, n), rows


def job(arg):
    name, v = arg
    import oracle
    cfg = CONFIGS[name]
    X, _ = synth.gaussian_sem(cfg["n"], cfg["N"], SEED)
    ds = oracle.Dataset(X)
    cands, _ = candidates(cfg, ds)
    t0 = time.time()
    sets, scores = ds.score_variable(LAM, v, cands[v], cfg["k"])
    dt = time.time() - t0
    order = np.argsort(sets, kind="stable")
    s, f = sets[order], scores[order]
    return name, v, {
        "candidates": int(cands[v]),
        "stored": int(len(s)),
        "sets_sha256": hashlib.sha256(s.astype(np.uint64).tobytes()).hexdigest(),
        "score_sum": float(np.sum(f.astype(np.float64))),
        "sample_sets": [int(x) for x in s[::STRIDE]],
        "sample_scores": [float(x) for x in f[::STRIDE]],
        "oracle_seconds": dt,
    }


def main():
    import oracle
    oracle.build()
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    path = os.path.join(ROOT, "tests", "golden", "c45_oracle.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    out = {"generator": "tests/golden/make_c45_fixture.py (oracle ora_score_variable, ora_mmpc)",
           "lambda": LAM, "seed": SEED, "sample_stride": STRIDE}
    for nm, c in CONFIGS.items():
        X, _ = synth.gaussian_sem(c["n"], c["N"], SEED)
        _, rows = candidates(c, oracle.Dataset(X))
        out[nm] = {k: v for k, v in c.items() if k != "variables"}
        out[nm]["skeleton_rows"] = rows
        kept = old.get(nm, {})
        same = kept.get("skeleton_rows") == rows and kept.get("k") == c["k"]
        out[nm]["per_variable"] = dict(kept.get("per_variable", {})) if same else {}
    jobs = [(nm, v) for nm, c in CONFIGS.items() for v in c["variables"]
            if str(v) not in out[nm]["per_variable"]]
    # Longest first (C5, then C4 by candidate count) so the pool ends together.
    X4, _ = synth.gaussian_sem(30, 100000, SEED)
    c4c, _ = candidates(CONFIGS["c4"], oracle.Dataset(X4))
    jobs.sort(key=lambda j: -(1 << 40) if j[0] == "c5" else -(1 << bin(c4c[j[1]]).count("1")))
    print(f"{len(jobs)} variables to run: {jobs}", flush=True)
    with Pool(procs) as p:
        for nm, v, res in p.imap_unordered(job, jobs):
            out[nm]["per_variable"][str(v)] = res
            print(f"{nm} v={v}: {res['stored']} stored in {res['oracle_seconds']:.0f} s", flush=True)
            json.dump(out, open(path + ".tmp", "w"), indent=1)
            os.replace(path + ".tmp", path)
    json.dump(out, open(path + ".tmp", "w"), indent=1)
    os.replace(path + ".tmp", path)
    print("wrote", path)


if __name__ == "__main__":
    main()
