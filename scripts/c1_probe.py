#!/usr/bin/env python3
"""C1 (data/hepatitis.clean.csv, -p 19) at one lambda: one scoring call with
the per-kernel profile (and, with ULG_WALK_STATS=1, the wide walks' step
statistics on stderr).

    python scripts/c1_probe.py [lambda] [--option name=value ...] [--digest out.json] [--no-profile]

--digest writes per-variable digests of the stored lists (count, sha256 of
the sets, score sum) so two walk forms can be compared on the layers the
oracle fixture does not reach."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "urlearning-cpp_amd"), os.path.join(ROOT, "tests")]
import ulg  # noqa: E402
from test_gpu_wide import load_csv_ascii  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lam", nargs="?", type=float, default=0.5)
ap.add_argument("--option", action="append", default=[])
ap.add_argument("--digest")
ap.add_argument("--no-profile", action="store_true")
args = ap.parse_args()

X = load_csv_ascii(os.path.join(ROOT, "tests", "golden", "hepatitis.clean.csv"))
n = X.shape[1]
ctx = ulg.Context(0)
for o in args.option:
    k, v = o.split("=")
    ctx.set_option(k, int(v))
ctx.load(X, args.lam)
ctx.profile(not args.no_profile)
t = time.perf_counter()
offs, sets, scores = ctx.score_all(list(range(n)), [(1 << n) - 1] * n, n - 1)
dt = time.perf_counter() - t
print(f"lambda {args.lam} {args.option}: {len(sets)} stored in {dt:.2f} s", flush=True)
if not args.no_profile:
    prof = ctx.profile_dump()
    for name, v in sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])[:12]:
        print(f"  {name:20s} {v['count']:5d} launches {v['total_ms']:10.1f} ms", flush=True)
if args.digest:
    per = []
    for v in range(n):
        s = np.ascontiguousarray(sets[offs[v]:offs[v + 1]], dtype=np.uint64)
        sc = scores[offs[v]:offs[v + 1]]
        per.append({"count": int(len(s)), "sets_sha256": hashlib.sha256(s.tobytes()).hexdigest(),
                    "scores_sha256": hashlib.sha256(np.ascontiguousarray(sc).tobytes()).hexdigest(),
                    "score_sum": float(sc.astype(np.float64).sum())})
    with open(args.digest, "w") as f:
        json.dump({"lambda": args.lam, "options": args.option, "seconds": dt, "per_variable": per}, f, indent=1)
