#!/usr/bin/env python3
"""Per-kernel average durations (us) of rocprofv3 kernel traces side by side,
keyed by kernel name and grid size: scripts/kab_table.py dir1 dir2 ...
(each dir holds a run_kernel_trace.csv, e.g. gpu_probe.sh's kab_<lib>/)."""
import collections
import csv
import glob
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        out[(k, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: sum(v) / len(v) for k, v in out.items()}, {k: len(v) for k, v in out.items()}


def main():
    runs = [load(d) for d in sys.argv[1:]]
    keys = sorted(set().union(*[r[0].keys() for r in runs]), key=lambda k: -max(r[0].get(k, 0) for r in runs))
    print(f"{'kernel':48s} {'grid':>9s} " + " ".join(f"{os.path.basename(os.path.dirname(d.rstrip('/')))[:10]:>10s}" for d in sys.argv[1:]))
    for k in keys[:int(os.environ.get("TOP", "30"))]:
        print(f"{k[0][:48]:48s} {k[1]:9d} " + " ".join(f"{r[0].get(k, float('nan')):10.1f}" for r in runs))


if __name__ == "__main__":
    main()
