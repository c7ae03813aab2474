"""HBM bytes of one GPU order-graph sweep (every layer_pull*_kernel dispatch
of the run -- round 6: the layer_pull_w32_kernel the sweep launches at C3,
search_gpu.hip -- divided by the number of sweeps = dispatches / n) from separate
FETCH_SIZE and WRITE_SIZE passes, corrected as MI355X_MICROARCH.md §HBM
prescribes for gfx950 (FETCH_SIZE doubled, WRITE_SIZE as is; both KiB).

  python scripts/pmc_search_summarize.py <fetch.csv> <write.csv> <config_id> <n> <out.json>
"""
import csv
import json
import math
import sys


def rows(path, counter):
    return [r for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and "layer_pull" in r["Kernel_Name"]]


def values(path, counter):
    return [float(r["Counter_Value"]) for r in rows(path, counter)]


def kernel_names(path, counter):
    return sorted({r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                   for r in rows(path, counter)})


def main():
    fetch_csv, write_csv, config_id, n, out = sys.argv[1:6]
    n = int(n)
    f, w = values(fetch_csv, "FETCH_SIZE"), values(write_csv, "WRITE_SIZE")
    if not f or not w or len(f) % n or len(w) % n:
        sys.exit(f"layer_pull_kernel dispatches {len(f)} / {len(w)} are not whole sweeps of {n}")
    sweeps_f, sweeps_w = len(f) // n, len(w) // n
    traffic = 2.0 * sum(f) * 1024.0 / sweeps_f + sum(w) * 1024.0 / sweeps_w
    # bench.py search_roofline: L predecessors x (4 B g + 4 B best-score cost) + 4 B g + 1 B leaf
    algo = sum(math.comb(n, L) * (8 * L + 5) for L in range(1, n + 1))
    names = kernel_names(fetch_csv, "FETCH_SIZE")
    res = {"kernel": names[0] if len(names) == 1 else names, "config_id": config_id, "n": n,
           "sweeps": [sweeps_f, sweeps_w],
           "fetch_kib_per_sweep": sum(f) / sweeps_f, "write_kib_per_sweep": sum(w) / sweeps_w,
           "traffic_bytes_per_sweep": traffic, "algorithmic_bytes_per_sweep": algo,
           "correction": "2 x FETCH_SIZE (gfx950 reports half of wide reads) + WRITE_SIZE",
           "sources": [fetch_csv, write_csv]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
