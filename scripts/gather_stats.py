#!/usr/bin/env python3
"""What the layer kernels' presence gathers find (a -DULG_GATHER_STATS build of
libulg.so): per (layer, phase), over the sets compacted for the gathers, the
hot children (P minus a member, or that plus variable 0, whose subset maximum
reaches -ts), and per set the keys read, present, >= -ts, and the keys the
hot-child rule and the cover rule would still have to read.

    python scripts/gather_stats.py --lib urlearning-cpp_amd/diag/libulg_stats.so [--cases c3 c5]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402
import synth  # noqa: E402
import ulg  # noqa: E402
from score_probe import CASES, cands_for  # noqa: E402

NAMES = ["sets", "hotA_children", "hotZ_children", "present", "hi", "need_hotsel", "hi_relevant", "cover",
         "present_and_need", "VIOL_hi_not_relevant", "VIOL_cover_not_need", "keys", "queued",
         "hi_relevant_or_cover", "present_not_need"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--cases", nargs="+", default=["c3", "c5"])
    a = ap.parse_args()
    ulg.LIB_PATH = os.path.abspath(a.lib)
    L_ = ulg.lib()
    L_.ulg_diag_gather_stats.argtypes = [C.c_void_p, C.c_void_p]
    ctx = ulg.Context(0)
    ctx.set_option("score_graph", 0)
    for name in a.cases:
        for (n, N, k, kind) in CASES[name]:
            X, _ = synth.gaussian_sem(n, N, 9200)
            ctx.load(X, 2.0)
            variables, cands = cands_for(n, kind, n)
            buf = np.zeros(2 * 2 * 9 * 16, dtype=np.uint64)
            L_.ulg_diag_gather_stats(ctx._h, buf.ctypes.data)  # zero
            st, scored = ctx.score(variables, cands, k)
            L_.ulg_diag_gather_stats(ctx._h, buf.ctypes.data)
            out = {"case": name, "n": n, "k": k, "stored": st, "scored": scored, "layers": {}}
            for L in range(1, 9):
                for ph in range(2):
                    c = buf[(L * 2 + ph) * 16:(L * 2 + ph) * 16 + 15]
                    if c[0] == 0:
                        continue
                    s = float(c[0])
                    out["layers"][f"L{L}p{ph}"] = dict({"sets": int(c[0])},
                                                        **{nm: round(float(v) / s, 3) for nm, v in
                                                           zip(NAMES[1:], c[1:])})
            wb = buf[2 * 9 * 16:]
            for L in range(1, 9):
                for ph in range(2):
                    w = wb[(L * 2 + ph) * 16:(L * 2 + ph) * 16 + 16]
                    if w.sum() == 0:
                        continue
                    out["layers"].setdefault(f"L{L}p{ph}", {})["walk_hits_by_depth"] = [int(x) for x in w[:L]]
                    out["layers"][f"L{L}p{ph}"]["walk_stored"] = int(w[15])
            print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
