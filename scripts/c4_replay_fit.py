#!/usr/bin/env python3
"""Split walk_wide_lds_kernel's counters into the fill (per local subset
filled) and the replay loop (per walk iteration): per dispatch of
scripts/r5_c4_pmc.sh's passes, counter = a * subsets_filled + b * iterations
+ c * blocks, least squares over the dispatches.  subsets_filled = blocks *
2^q; iterations = the completed replays' (ULG_WALK_STATS) plus the host
budget for each replay handed to the host (512 for launches of <= 64
replays, else 1024).

    python scripts/c4_replay_fit.py gpurun_out/r5c4pmc > profiles/r5/c4_replay_fit.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

import numpy as np


def main():
    d = sys.argv[1]
    out = {"model": "counter = a * subsets_filled + b * iterations + c * blocks (least squares over dispatches)",
           "source": d, "passes": {}}
    for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        log = os.path.join(d, os.path.basename(os.path.dirname(p)) + ".log")
        stats = [dict(L=int(m[0]), ph=int(m[1]), q=int(m[2]), rep=int(m[3]), it=int(m[4]))
                 for m in re.findall(r"walk_lds_stats L=(\d+) phase=(\d) q=(\d+) replays=(\d+) iters=(\d+)", open(log).read())]
        disp = collections.OrderedDict()
        for r in csv.DictReader(open(p)):
            if "walk_wide_lds_kernel" not in r["Kernel_Name"]:
                continue
            e = disp.setdefault(int(r["Dispatch_Id"]), {"blocks": int(r["Grid_Size"]) // int(r["Workgroup_Size"]),
                                                       "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
        ds = [disp[k] for k in sorted(disp)]
        if len(ds) != len(stats):
            out["passes"][p] = f"dispatches {len(ds)} != stats lines {len(stats)}"
            continue
        X, rows = [], []
        for e, s in zip(ds, stats):
            bud = 512 if e["blocks"] <= 64 else 1024
            iters = s["it"] + (e["blocks"] - s["rep"]) * bud if e["blocks"] <= 4096 else s["it"]
            X.append([e["blocks"] * (1 << s["q"]), iters, e["blocks"]])
            rows.append(dict(L=s["L"], phase=s["ph"], q=s["q"], blocks=e["blocks"], iterations=iters,
                             duration_us=e["ns"] / 1e3))
        X = np.array(X, dtype=float)
        fit = {}
        for cn in [k for k in ds[0] if k.startswith("SQ_")]:
            y = np.array([e[cn] for e in ds])
            coef, res, rank, _ = np.linalg.lstsq(X, y, rcond=None)
            pred = X @ coef
            r2 = 1 - ((y - pred) ** 2).sum() / max(((y - y.mean()) ** 2).sum(), 1e-30)
            fit[cn] = {"per_subset_filled": coef[0], "per_iteration": coef[1], "per_block": coef[2], "r2": r2}
        out["passes"][os.path.basename(os.path.dirname(p))] = {"fit": fit, "dispatches": rows}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
