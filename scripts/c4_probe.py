#!/usr/bin/env python3
"""C4 (n=30, N=100k, MMPC skeleton, 2-hop candidates, -p = n-1) scored one
variable at a time on the GPU, smallest candidate set first, printing the
time of each so a slow variable shows up before the whole call would.

    python scripts/c4_probe.py [max_parents] [variables...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 29
    n, N = 30, 100000
    X, _ = synth.gaussian_sem(n, N, 9200)
    ctx = ulg.Context(0)
    for kv in filter(None, os.environ.get("ULG_OPTS", "").split(",")):  # A/B knobs: name=value,...
        a, b = kv.split("=")
        ctx.set_option(a, int(b))
    ctx.load(X, 2.0)
    rows = ctx.mmpc(0.01)
    cands = ulg.candidates_from_edges(rows, n)
    m = [bin(c & ~(1 << v)).count("1") for v, c in enumerate(cands)]
    vs = [int(a) for a in sys.argv[2:]] or sorted(range(n), key=lambda v: m[v])
    total = 0.0
    for v in vs:
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        stored, scored = ctx.score([v], [cands[v]], k)
        dt = time.perf_counter() - t0
        prof = ctx.profile_dump()
        ctx.profile(False)
        total += dt
        top = sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])[:4]
        print(f"v={v:2d} m={m[v]:2d} scored={scored:8d} stored={stored:7d} {dt * 1e3:9.1f} ms  "
              + " ".join(f"{a}={b['total_ms']:.1f}" for a, b in top), flush=True)
    print(f"total {total:.2f} s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
