"""Generate tests/golden/c1_hepatitis_digest.json: the CPU oracle's score run
of config C1 (data/hepatitis.clean.csv, the reference's default -p = n-1 = 19,
full skeleton) reduced to a per-variable digest, so that the GPU test can
check all 10.5 M scored sets without re-running the oracle on the GPU box
(lambda 2: about 20 s on 8 threads; lambda <= 1 leaves far more large sets
for the find_best_subset_score recursion and runs past 10 minutes, so the
fixture holds lambda 2, the README's usage).

Per variable: the stored count, the SHA-256 of the stored sets (uint64, in
(|set|, set) order -- bit-exact index work), the float64 sum of the stored
scores, and 64 (set, score) samples at fixed list positions (1e-6 relative).

Run from the repo root:  python tests/golden/make_c1_digest.py [lambda ...]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

CSV = os.path.join(ROOT, "tests", "golden", "hepatitis.clean.csv")
SAMPLES = 64


def digest(offs, sets, scores, n):
    out = []
    for v in range(n):
        s = sets[offs[v]:offs[v + 1]]
        sc = scores[offs[v]:offs[v + 1]]
        pos = np.unique(np.linspace(0, len(s) - 1, SAMPLES).astype(np.int64)) if len(s) else np.zeros(0, np.int64)
        out.append({
            "count": int(len(s)),
            "sets_sha256": hashlib.sha256(np.ascontiguousarray(s, dtype=np.uint64).tobytes()).hexdigest(),
            "score_sum": float(sc.astype(np.float64).sum()),
            "samples": [[int(s[p]), float(sc[p])] for p in pos],
        })
    return out


def main(lams):
    ds = oracle.Dataset(csv_path=CSV)
    n = ds.n
    out = os.path.join(ROOT, "tests", "golden", "c1_hepatitis_digest.json")
    res = {"csv": "hepatitis.clean.csv", "n": n, "N": int(ds.N), "max_parents": n - 1, "runs": {}}
    if os.path.exists(out):  # add to the lambdas already there
        with open(out) as f:
            res["runs"].update(json.load(f)["runs"])
    for lam in lams:
        offs, sets, scores = ds.score_all(lam, [(1 << n) - 1] * n, n - 1, threads=os.cpu_count() or 8)
        res["runs"][repr(float(lam))] = digest(offs, sets, scores, n)
        print(f"lambda={lam}: {int(offs[n])} stored sets", flush=True)
        with open(out, "w") as f:  # after every lambda: a long run keeps what it finished
            json.dump(res, f, indent=0)


if __name__ == "__main__":
    main([float(x) for x in sys.argv[1:]] or [2.0])
