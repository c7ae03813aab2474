"""Generate tests/golden/c1_hepatitis_default.json: config C1 at the
reference's defaults -- data/hepatitis.clean.csv, lambda 0.5
(score/score_main.cpp:214) and -p n - 1 = 19 (:296-298).

The oracle's literal find_best_subset_score recursion cannot finish the 19
layers at lambda 0.5 (hours), but a layer's stored sets depend only on the
layers below it (score_calculator.cpp:83-120), so the oracle run with
-p K pins layers 1..K of the -p 19 run exactly.  Per variable: the count, the
SHA-256 of the stored sets in (|set|, set) order, the float64 score sum and
64 (set, score) samples (digest() of make_c1_digest.py).

Run from the repo root (about 20 min on 8 threads for K = 12):
    python tests/golden/make_c1_default_fixture.py [K]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")]
import oracle  # noqa: E402
from make_c1_digest import CSV, digest  # noqa: E402

LAM = 0.5


def main(K):
    import time
    ds = oracle.Dataset(csv_path=CSV)
    n = ds.n
    t0 = time.time()
    offs, sets, scores = ds.score_all(LAM, [(1 << n) - 1] * n, K, threads=os.cpu_count() or 8)
    res = {"csv": "hepatitis.clean.csv", "n": n, "N": int(ds.N), "lambda": LAM, "max_parents_run": n - 1,
           "layers_checked": K, "oracle_seconds": time.time() - t0,
           "generator": "tests/golden/make_c1_default_fixture.py (oracle ora_score_all, -p K)",
           "per_variable": digest(offs, sets, scores, n)}
    with open(os.path.join(ROOT, "tests", "golden", "c1_hepatitis_default.json"), "w") as f:
        json.dump(res, f, indent=0)
    print(f"K={K}: {int(offs[n])} stored sets in {res['oracle_seconds']:.0f} s", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 12)
