"""Config C1 (hepatitis, default -p 19) on the GPU at several lambdas: the
wide layers' walk load grows as lambda shrinks (more large sets survive)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ulg
from test_gpu_wide import load_csv_ascii
X = load_csv_ascii(os.path.join(ROOT, "tests", "golden", "hepatitis.clean.csv"))
n = X.shape[1]
ctx = ulg.Context(0)
ctx.profile(True)
for lam in [float(x) for x in sys.argv[1:]] or [2.0, 1.0, 0.5]:
    ctx.load(X, lam)
    ctx.profile_reset()
    t0 = time.perf_counter()
    st, sc = ctx.score(list(range(n)), [(1 << n) - 1] * n, n - 1)
    dt = time.perf_counter() - t0
    prof = ctx.profile_dump()
    top = sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])[:4]
    print(f"lambda={lam}: {sc} scored, {st} stored in {dt:.3f} s; " +
          ", ".join(f"{k} {v['total_ms']:.1f} ms" for k, v in top), flush=True)
