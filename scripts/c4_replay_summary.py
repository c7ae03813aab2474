#!/usr/bin/env python3
"""Instructions and wave cycles per replay iteration of walk_wide_lds_kernel
from scripts/r5_c4_pmc.sh's passes (each pass's log carries ULG_WALK_STATS'
per-launch iteration counts; the counters are summed over the same
launches).

    python scripts/c4_replay_summary.py gpurun_out/r5c4pmc
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    out = {}
    for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        log = os.path.join(d, os.path.basename(os.path.dirname(p)) + ".log")
        iters = sum(int(m.group(1)) for m in re.finditer(r"walk_lds_stats .* iters=(\d+)", open(log).read()))
        replays = sum(int(m.group(1)) for m in re.finditer(r"walk_lds_stats .* replays=(\d+)", open(log).read()))
        tot = collections.defaultdict(float)
        disp = set()
        for r in csv.DictReader(open(p)):
            if "walk_wide_lds_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        out["iterations"], out["replays"], out["dispatches"] = iters, replays, len(disp)
        for c, v in tot.items():
            out[c + "_per_iteration"] = v / max(iters, 1)
    # SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_ACTIVE_* count in quad-cycles (x4 = shader cycles)
    if "SQ_WAVE_CYCLES_per_iteration" in out:
        out["note"] = ("per GPU replay iteration over every walk_wide_lds_kernel launch of the run; the wave-cycle "
                       "counters (SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_ACTIVE_*, SQ_BUSY_CYCLES) are in units of 4 "
                       "cycles and include the fill waves (waves 1-3 of 256-thread launches)")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
