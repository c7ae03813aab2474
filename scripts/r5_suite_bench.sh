#!/bin/bash
# The whole GPU suite, smoke(), then the default bench line (round-end shape).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5suite}
mkdir -p $OUT
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
head -c 400 $OUT/bench.json
