#!/bin/bash
# A/B of the bit-sliced walk's sets per lane (ULG_SLICED_K) at C3: one short
# bench per setting, scoring only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in ${KS:-"2,4" "2,8" "4,4" "4,8" "8,8" "1"}; do
  ULG_SLICED_K=$k timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-search > gpurun_out/absk.json 2>/dev/null || exit $?
  python - "$k" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/absk.json").read())
km = d["kernel_ms_one_step"]
print(f"K={sys.argv[1]:4s} step {d['ms_per_step']:.3f} ms  walk6 rest/var0 {km.get('walk_6_rest', 0):.3f}/{km.get('walk_6_var0', 0):.3f}  walk5 {km.get('walk_5_rest', 0):.3f}/{km.get('walk_5_var0', 0):.3f}", flush=True)
PY
done
