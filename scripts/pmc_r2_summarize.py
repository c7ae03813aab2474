#!/usr/bin/env python3
"""Summarise scripts/pmc_r2.sh: (1) the FETCH_SIZE calibration on the known-
byte kernels of scripts/gather_probe.hip, (2) per-launch read/write traffic
of the scorer's roofline pair and of the GPU sweep from the bench passes,
with the calibrated read factor applied, (3) the SQ pass of the scorer pair.

  python scripts/pmc_r2_summarize.py gpurun_out/pmc2 profiles/r2
"""
import csv
import glob
import json
import math
import os
import shutil
import sys
from collections import defaultdict


def rows(d, name):
    f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))
    return list(csv.DictReader(open(f[0]))) if f else []


def per_dispatch(rs):
    """{dispatch_id: (kernel, {counter: value})} in dispatch order"""
    out = {}
    for r in rs:
        k = int(r["Dispatch_Id"])
        out.setdefault(k, (r["Kernel_Name"], {}))[1][r["Counter_Name"]] = float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


PROBE_KNOWN = ["stream16", "gather4_hbm", "gather8_hbm", "gather4_mall_warm", "gather4_mall", "run4_hbm"]


def probe(d):
    passes = {p: [x for x in per_dispatch(rows(d, p)) if "rocclr" not in x[0]] for p in ("g_fetch", "g_req", "g_dram")}
    log = open(os.path.join(d, "g_fetch.log")).read()
    line = next(ln for ln in log.splitlines() if ln.startswith("{\"launches\""))
    known = json.loads(line.replace("}{", "}, {"))  # first probe build printed no commas
    res = []
    for i, name in enumerate(PROBE_KNOWN):
        kb = known["launches"][i]["known_read_bytes"]
        c = {}
        for p in passes.values():
            c.update(p[i][1])
        fetch = c["FETCH_SIZE"] * 1024
        e = {"launch": name, "known_read_bytes": kb, "fetch_size_bytes": fetch, "fetch_over_known": fetch / kb,
             "rdreq": c.get("TCC_EA0_RDREQ_sum"), "rdreq_32b": c.get("TCC_EA0_RDREQ_32B_sum"),
             "bubble_128b": c.get("TCC_BUBBLE_sum"), "rdreq_dram": c.get("TCC_EA0_RDREQ_DRAM_sum"),
             "rdreq_dram_32b": c.get("TCC_EA0_RDREQ_DRAM_32B_sum"), "ms": known["launches"][i]["ms"]}
        if name != "stream16" and name != "run4_hbm":
            n = known["gather_count"]
            e["fetch_bytes_per_access"] = fetch / n
            e["rdreq_per_access"] = (c.get("TCC_EA0_RDREQ_sum") or 0) / n
            e["dram_req_per_access"] = (c.get("TCC_EA0_RDREQ_DRAM_sum") or 0) / n
        res.append(e)
    return res


def group(dispatches, pred):
    sel = [c for k, c in dispatches if pred(k)]
    tot = defaultdict(float)
    for c in sel:
        for a, b in c.items():
            tot[a] += b
    return len(sel), {a: b / max(1, len(sel)) for a, b in tot.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    cal = probe(d)
    bench = {p: per_dispatch(rows(d, p)) for p in ("b_fetch", "b_write", "b_req", "b_dram", "b_sq")}
    kernels = {
        "score_layer_6_rest": lambda k: k.startswith("void (anonymous namespace)::score_layer_kernel<6, 1"),
        "walk_6_rest": lambda k: "walk_sliced_kernel<6, 1" in k,
        "layer_pull_kernel(sweep table)": lambda k: "layer_pull_w32_kernel" in k,
    }
    per = {}
    for nm, pred in kernels.items():
        e = {}
        for p, ds in bench.items():
            cnt, avg = group(ds, pred)
            e["dispatches_" + p] = cnt
            e.update(avg)
        per[nm] = e
    # gather calibration: random 4 B reads (the scorer's slab gathers, the
    # sweep's g / cost reads) -- FETCH_SIZE bytes per access measured on
    # distinct-line gathers
    g4 = next(x for x in cal if x["launch"] == "gather4_hbm")
    s16 = next(x for x in cal if x["launch"] == "stream16")
    res = {"calibration": cal,
           "factor_stream16": s16["known_read_bytes"] / s16["fetch_size_bytes"],
           "gather4_fetch_bytes_per_access": g4["fetch_bytes_per_access"],
           "kernels": per}
    json.dump(res, open(os.path.join(out, "pmc_r2.json"), "w"), indent=1)
    for p in ("g_fetch", "g_req", "g_dram", "b_fetch", "b_write", "b_req", "b_dram", "b_sq"):
        for f in glob.glob(os.path.join(d, p, "*counter_collection.csv")):
            shutil.copy(f, os.path.join(out, f"pmc_{p}.csv"))
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    for k, v in per.items():
        print(k, {a: (round(b, 1) if isinstance(b, float) else b) for a, b in v.items()})


if __name__ == "__main__":
    main()


def bench_traffic(summary_path, out_dir):
    """profiles/r2/pmc_traffic.json and pmc_search_traffic.json in the form
    bench.py reads: read bytes = 2 x FETCH_SIZE (every TCC->EA read request of
    these kernels is a 128 B line tallied as 64 B: gather_probe's 4 B and 8 B
    random gathers and 64-lane runs all show RDREQ x 128 B = 2 x FETCH_SIZE =
    4 x 32 B DRAM-side units) + WRITE_SIZE.  Infinity-Cache hits are counted
    (gather4_mall), so this is L2-miss traffic, an upper bound on HBM bytes."""
    res = json.load(open(summary_path))
    k = res["kernels"]
    a, b = k["score_layer_6_rest"], k["walk_6_rest"]
    pair = 2 * 1024 * (a["FETCH_SIZE"] + b["FETCH_SIZE"]) + 1024 * (a["WRITE_SIZE"] + b["WRITE_SIZE"])
    note = ("2 x FETCH_SIZE + WRITE_SIZE; the x2 is calibrated for this repo's access patterns by "
            "scripts/gather_probe.hip (profiles/r2/pmc_r2.json: random 4 B / 8 B gathers and 64-lane runs "
            "fetch one 128 B line per TCC read request, FETCH_SIZE tallies 64 B); Infinity-Cache hits included")
    json.dump({"kernel": "score_layer_kernel<6, 1,;walk_sliced_kernel<6, 1,", "label": "score_layer_6_rest + walk_6_rest",
               "config_id": "c3", "sets_per_launch": 852441,
               "dispatches": [a["dispatches_b_fetch"], a["dispatches_b_write"]],
               "fetch_kib_avg": a["FETCH_SIZE"] + b["FETCH_SIZE"], "write_kib_avg": a["WRITE_SIZE"] + b["WRITE_SIZE"],
               "traffic_bytes_per_launch": pair, "correction": note,
               "sources": ["profiles/r2/pmc_b_fetch.csv", "profiles/r2/pmc_b_write.csv"]},
              open(os.path.join(out_dir, "pmc_traffic.json"), "w"), indent=1)
    p = k["layer_pull_kernel(sweep table)"]
    n = 25
    sweeps = p["dispatches_b_fetch"] // n
    per_sweep = n * (2 * 1024 * p["FETCH_SIZE"] + 1024 * p["WRITE_SIZE"])
    algo = sum(math.comb(n, L) * (8 * L + 5) for L in range(1, n + 1))
    json.dump({"kernel": "layer_pull_w32_kernel", "config_id": "c3", "n": n, "sweeps": sweeps,
               "fetch_kib_per_sweep": n * p["FETCH_SIZE"], "write_kib_per_sweep": n * p["WRITE_SIZE"],
               "traffic_bytes_per_sweep": per_sweep, "algorithmic_bytes_per_sweep": algo,
               "correction": note, "sources": ["profiles/r2/pmc_b_fetch.csv", "profiles/r2/pmc_b_write.csv"]},
              open(os.path.join(out_dir, "pmc_search_traffic.json"), "w"), indent=1)
    print("pair traffic", pair, "sweep traffic", per_sweep, "algo", algo)


if len(sys.argv) > 3 and sys.argv[3] == "--bench-traffic":
    bench_traffic(os.path.join(sys.argv[2], "pmc_r2.json"), sys.argv[2])
