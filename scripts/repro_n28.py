"""n = 28, k = 3, full skeleton: score, then build the best-score tables
(ulg_search_from_scores) -- the launch that failed with 'invalid
configuration argument' in test_table_sharded_sweep_equals_single_gpu."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "urlearning-cpp_amd"))
import synth  # noqa: E402
import ulg  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
X, _ = synth.gaussian_sem(n, 5000, 9761)
ctx = ulg.Context(0)
ctx.load(X, 2.0)
print(ctx.score(list(range(n)), [(1 << n) - 1] * n, 3), flush=True)
ctx.search_from_scores()
print("tables ok", flush=True)
