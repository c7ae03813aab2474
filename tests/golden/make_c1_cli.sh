#!/bin/bash
# Config C1 through the oracle's command lines (oracle/build/ref_score,
# ref_astar): data/hepatitis.clean.csv, cBIC, --lambda 2, full 20x20 skeleton,
# default -p (n - 1 = 19).  Records the .pss SHA-256 / size and the netFile /
# netFile.csv text in tests/golden/c1_hepatitis_cli.json for the GPU CLI test
# (the oracle needs about 3.5 CPU-minutes for this, the GPU box does not re-run it).
# Run from the repo root after `make -C oracle`.
set -euo pipefail
D=$(cd "$(dirname "$0")" && pwd)
W=$(mktemp -d)
python3 -c "print('\n'.join([','.join(['1'] * 20)] * 20))" > "$W/full20.csv"
R=$(pwd)
# relative input path: the .pss header records it (META input_file)
(cd "$D" && "$R/oracle/build/ref_score" hepatitis.clean.csv "$W/c1.pss" -f cBIC --lambda 2 -k "$W/full20.csv")
oracle/build/ref_astar "$W/c1.pss" -k "$W/full20.csv" -n "$W/net" | grep "Found solution" > "$W/solution"
python3 - "$W" "$D/c1_hepatitis_cli.json" <<'PY'
import hashlib, json, os, sys
w, out = sys.argv[1], sys.argv[2]
h = hashlib.sha256()
with open(os.path.join(w, "c1.pss"), "rb") as f:
    for chunk in iter(lambda: f.read(1 << 24), b""):
        h.update(chunk)
json.dump({"csv": "hepatitis.clean.csv", "lambda": "2", "skeleton": "full 20x20 ones",
           "pss_sha256": h.hexdigest(), "pss_bytes": os.path.getsize(os.path.join(w, "c1.pss")),
           "net": open(os.path.join(w, "net")).read(), "net_csv": open(os.path.join(w, "net.csv")).read(),
           "solution": open(os.path.join(w, "solution")).read().strip()},
          open(out, "w"), indent=1)
PY
rm -rf "$W"
