#!/usr/bin/env python3
"""Average duration per (kernel, grid size) of each build in a
scripts/r5_kernel_ab.sh output directory, side by side.

    python scripts/kernel_ab_table.py gpurun_out/r5kab [kernel substrings...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    pats = sys.argv[2:] or ["score_layer_kernel<6", "walk_sliced_kernel<6", "score_layer_kernel<5", "walk_sliced_kernel<5"]
    res = collections.defaultdict(dict)
    builds = []
    for f in sorted(glob.glob(os.path.join(d, "*", "run_kernel_trace.csv"))):
        b = f.split(os.sep)[-2]
        builds.append(b)
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if any(p in n for p in pats):
                key = (n.split("(")[1][:-2] if False else n[n.find("::") + 2:n.find(">(") + 1], r.get("Grid_Size", r.get("Grid_Size_X")))
                acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in acc.items():
            v.sort()
            res[k][b] = (sum(v) / len(v), v[len(v) // 2], len(v))
    print("%-40s %9s " % ("kernel", "grid") + " ".join("%22s" % b for b in builds))
    for k in sorted(res, key=lambda x: (x[0], -int(x[1]))):
        print("%-40s %9s " % k + " ".join("%10.1f/%5.1f(%3d)" % res[k][b] if b in res[k] else "%22s" % "-" for b in builds))


if __name__ == "__main__":
    main()
