#!/usr/bin/env python3
"""Per-wave timing of the bit-sliced walk launches (ULG_WALK_CLOCK): one C3
call on one stream, then for each layer/phase the kernel span, the wave
duration quantiles and the union points of the slowest waves.

    python scripts/walk_clock.py [--case c3|c5] [--out gpurun_out/wclock]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="c3")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wclock"))
    ap.add_argument("--options", default="", help="name=value,... (ulg_set_option)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    os.environ["ULG_WALK_CLOCK"] = a.out
    import numpy as np
    import synth
    import ulg
    n, N = (25, 10000) if a.case == "c3" else (32, 50000)
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx = ulg.Context(0)
    ctx.set_option("score_streams", 1)
    for kv in filter(None, a.options.split(",")):
        k_, v_ = kv.split("=")
        ctx.set_option(k_, int(v_))
    ctx.load(X, 2.0)
    full = (1 << n) - 1
    ctx.score(list(range(n)), [full] * n, 6)
    for L in range(1, 7):
        for ph in (0, 1):
            fn = os.path.join(a.out, f"sliced_L{L}_p{ph}.bin")
            if not os.path.exists(fn):
                continue
            w = np.fromfile(fn, dtype=np.uint64).reshape(-1, 3)
            w = w[w[:, 1] > 0]
            if len(w) == 0:
                continue
            st, en, pts = w[:, 0].astype(np.int64), w[:, 1].astype(np.int64), w[:, 2]
            d = (en - st) / 100.0  # 100 MHz wall clock: us
            span = (en.max() - st.min()) / 100.0
            q = np.percentile(d, [50, 90, 99, 100])
            top = np.argsort(-d)[:5]
            print(f"L{L} p{ph}: waves={len(w)} span_us={span:.1f} dur_us p50={q[0]:.1f} p90={q[1]:.1f} "
                  f"p99={q[2]:.1f} max={q[3]:.1f} sum_us={d.sum():.0f} | slowest: "
                  + ", ".join(f"{d[i]:.1f}us/{int(pts[i])}pts@{(st[i] - st.min()) / 100.0:.0f}" for i in top),
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
