"""Per-launch HBM traffic of one kernel from separate rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE each in its own pass, MI355X_MICROARCH.md
§rocprofv3 PMC slots), corrected as §HBM prescribes for gfx950: FETCH_SIZE
reports half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE
is taken as is.  Both are in KiB per dispatch.

  python scripts/pmc_summarize.py <fetch_pass.csv> <write_pass.csv> <kernel substrings, ";"-separated> \
      <config_id> <sets_per_launch> <out.json> [label]

With several kernels (the scoring kernel and the walk kernel of one layer),
the per-dispatch averages are summed: one layer launch = one dispatch of each.
"""
import csv
import json
import sys


def per_dispatch(path, counter, kernel):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, kernels, config_id, sets, out = sys.argv[1:7]
    label = sys.argv[7] if len(sys.argv) > 7 else kernels
    fetch_kib = write_kib = 0.0
    disp = []
    for kernel in kernels.split(";"):
        f = per_dispatch(fetch_csv, "FETCH_SIZE", kernel)
        w = per_dispatch(write_csv, "WRITE_SIZE", kernel)
        if not f or not w:
            sys.exit(f"no {kernel} dispatches with FETCH_SIZE/WRITE_SIZE in {fetch_csv} / {write_csv}")
        fetch_kib += sum(f) / len(f)
        write_kib += sum(w) / len(w)
        disp.append([len(f), len(w)])
    traffic = 2.0 * fetch_kib * 1024.0 + write_kib * 1024.0
    res = {"kernel": kernels, "label": label, "config_id": config_id, "sets_per_launch": int(sets),
           "dispatches": disp,
           "fetch_kib_avg": fetch_kib, "write_kib_avg": write_kib, "traffic_bytes_per_launch": traffic,
           "correction": "2 x FETCH_SIZE (gfx950 reports half of wide reads) + WRITE_SIZE",
           "sources": [fetch_csv, write_csv]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
