#!/usr/bin/env python3
"""Per-call kernel times of a score_probe.py kernel trace (gpu_probe.sh kab):
calls split at call_prologue_kernel; per case (the probe's --cases in order,
--reps + 2 calls each) the median call span and each kernel's average.

    python scripts/kab_calls.py <kab dir> [cases...] [--reps 5] [--match walk,score_layer]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("cases", nargs="*", default=["c3", "c5"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--match", default="walk,score_layer")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if k.startswith("call_prologue"):
            cur = []
            calls.append(cur)
        if cur is not None:
            cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    per = a.reps + 2
    pats = a.match.split(",")
    for ci, name in enumerate(a.cases):
        cs = calls[ci * per + 1: ci * per + per - 1]
        spans = sorted((c[-1][2] - c[0][1]) / 1e3 for c in cs)
        agg = collections.defaultdict(list)
        for c in cs:
            for k, s, e in c:
                agg[k].append((e - s) / 1e3)
        print(f"{name}: call span median {spans[len(spans) // 2]:.1f} us")
        for k, v in agg.items():
            if any(p in k for p in pats):
                print(f"   {k:45s} {sum(v) / len(v):8.1f}  x{len(v) // max(len(cs), 1)}")


if __name__ == "__main__":
    main()
