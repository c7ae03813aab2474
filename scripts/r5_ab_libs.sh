#!/bin/bash
# A/B of libulg.so builds (LIBS, space-separated) on single calls, alternating
# over two rounds, with the same options (OPTS): digests must agree; times
# side by side.  WCLOCK=<options> adds a per-wave walk-clock pass per build.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p $OUT
for rep in 1 2; do
  for lib in ${LIBS}; do
    nm=$(basename $lib .so)
    timeout -k 10 240 python3 scripts/score_probe.py --lib $lib --cases ${CASES:-c3 c5} --reps 10 --options ${OPTS:-score_streams=3} > $OUT/${nm}_${rep}.log 2>&1
  done
done
if [ -n "${WCLOCK:-}" ]; then
  for lib in ${LIBS}; do
    nm=$(basename $lib .so)
    ULG_LIB=$lib timeout -k 10 120 python3 scripts/walk_clock.py --case c3 --options ${WCLOCK} --out $OUT/wc_$nm > $OUT/wclock_$nm.log 2>&1
  done
fi
echo ab ok
