#!/usr/bin/env python3
"""Per-dispatch counters of the scorer's roofline pair from a
scripts/gpu_probe.sh pmc_scorer output directory: layer 6 without variable 0
at C3, score_layer_kernel<6, 1, 209> (grid = the layer's 2,557,324 sets
rounded to 256) plus walk_bucket_kernel<6, 1, K> (round 5: <6, 1, 81> and
walk_sliced_kernel<6, 1, K>).

* traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB per dispatch, gfx950
  correction of MI355X_MICROARCH.md, calibrated for gathers in
  DESIGN.md §3) -- per launch pair;
* l1_lines_per_set = TCP_TOTAL_CACHE_ACCESSES / sets (vector L1 tag lookups:
  a divergent 4-byte gather costs one per distinct 128-byte line per lane);
* ta_busy_frac = (TA_TA_BUSY_sum / 256 CUs) / (GRBM_GUI_ACTIVE / 8 XCDs):
  the fraction of the kernel's cycles the average CU's texture-address unit
  is busy.

    python scripts/pmc_r5_summarize.py gpurun_out/<tag> > profiles/r6/pmc_scorer.json
"""
import csv
import glob
import json
import os
import subprocess
import sys

# (kernel name prefix; the dispatches averaged are those with the largest
# grid, i.e. the full-layer launches of one stream per context)
# round 6: variant 241 (V = 209) and the key-sorted walk (walk_bucket_kernel;
# its count / scatter kernels are summed in as "sort" when present)
KERNELS = {"score": "score_layer_kernel<6, 1, 209>", "walk": "walk_bucket_kernel<6, 1, "}
N_CU, N_XCD = 256, 8


def per_dispatch(outdir):
    vals = {k: {} for k in KERNELS}
    files = sorted(glob.glob(os.path.join(outdir, "p*", "run_counter_collection.csv")))
    grid = {k: 0 for k in KERNELS}
    names = {k: None for k in KERNELS}
    for p in files:
        for r in csv.DictReader(open(p)):
            for k, name in KERNELS.items():
                if name in r["Kernel_Name"] and int(r["Grid_Size"]) > grid[k]:
                    grid[k] = int(r["Grid_Size"])
                    names[k] = r["Kernel_Name"].split("(")[1].rstrip(")") if False else r["Kernel_Name"][
                        r["Kernel_Name"].find("::") + 2:r["Kernel_Name"].find(">(") + 1]
    for p in files:
        for r in csv.DictReader(open(p)):
            for k, name in KERNELS.items():
                if name in r["Kernel_Name"] and int(r["Grid_Size"]) == grid[k]:
                    vals[k].setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"] + p, 0.0)
                    vals[k][r["Counter_Name"]][r["Dispatch_Id"] + p] += float(r["Counter_Value"])
    out = {k: {c: sum(d.values()) / len(d) for c, d in v.items()} | {"dispatches": {c: len(d) for c, d in v.items()}}
           for k, v in vals.items()}
    for k in KERNELS:
        out[k]["kernel"], out[k]["grid"] = names[k], grid[k]
    return out


def main():
    outdir = sys.argv[1]
    sets = 2557324
    pd = per_dispatch(outdir)
    out = {"config_id": "c3", "label": "score_layer_6_rest + walk_6_rest", "sets_per_launch": sets,
           "kernels": {k: pd[k]["kernel"] for k in KERNELS}, "grids": {k: pd[k]["grid"] for k in KERNELS},
           "source": outdir}
    try:
        out["commit"] = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                       cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip() or None
    except OSError:
        out["commit"] = None
    tr, l1 = 0.0, 0.0
    for k in KERNELS:
        c = pd[k]
        e = {}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["traffic_bytes"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            tr += e["traffic_bytes"]
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
            e["l1_lines_per_set"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"] / sets
            l1 += e["l1_lines_per_set"]
        if "TA_TA_BUSY_sum" in c and c.get("GRBM_GUI_ACTIVE"):
            e["ta_busy_frac"] = (c["TA_TA_BUSY_sum"] / N_CU) / (c["GRBM_GUI_ACTIVE"] / N_XCD)
            e["kernel_cycles_per_xcd"] = c["GRBM_GUI_ACTIVE"] / N_XCD
        # VALU instructions per wave, and resident waves per SIMD over the
        # kernel (SQ_WAVE_CYCLES counts quad-cycles: x4 cycles, / 4 SIMDs per CU)
        if c.get("SQ_WAVES"):
            e["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_WAVES"]
            e["salu_per_wave"] = c.get("SQ_INSTS_SALU", 0.0) / c["SQ_WAVES"]
        if "SQ_WAVE_CYCLES" in c and e.get("kernel_cycles_per_xcd"):
            e["resident_waves_per_simd"] = c["SQ_WAVE_CYCLES"] / (e["kernel_cycles_per_xcd"] * N_CU)
        if "TCP_TCC_READ_REQ_sum" in c and c["TCP_TCC_READ_REQ_sum"]:
            e["l1_to_l2_latency_cycles"] = c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"]
        e["counters_per_dispatch"] = {kk: round(vv, 1) for kk, vv in c.items()
                                      if kk not in ("dispatches", "kernel", "grid")}
        e["dispatches_averaged"] = c.get("dispatches", {})
        out[k] = e
    out["traffic_bytes_per_launch"] = tr or None
    out["l1_lines_per_set"] = l1 or None
    out["ta_busy_frac"] = out["score"].get("ta_busy_frac")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
