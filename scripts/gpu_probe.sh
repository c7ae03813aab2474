#!/bin/bash
# One GPU-box driver for every measurement this repo takes (round 6: it
# replaces round 5's scripts/r5_*.sh and r4_probe.sh).  STEPS picks the steps,
# in order; every GPU step runs under its own time limit and the first failure
# ends the script (set -e), so a fault or hang starts nothing more.
#
#   STEPS="suite smoke bench" TAG=r6a bash scripts/gpu_probe.sh
#
# steps (outputs under gpurun_out/$TAG):
#   suite       pytest -m gpu (PYTEST_ARGS, e.g. a file list / -k)
#   smoke       __graft_entry__.smoke()
#   bench       the default bench line (BENCH_ARGS)            -> bench.json
#   trace       rocprofv3 --kernel-trace --stats of that bench  -> trace/
#   pmc_scorer  FETCH / WRITE / TA-TCP / two SQ passes of the bench's timed
#               configuration, summarised (pmc_r5_summarize.py) -> pmc_scorer.json
#   pmc_search  FETCH / WRITE passes of a C3 bench with the search side,
#               summarised for the sweep kernel                -> pmc_search_traffic.json
#   probe       scripts/score_probe.py per build in LIBS (default the shipped
#               one), CASES, OPTS, two alternating rounds      -> probe_<lib>_<rep>.log
#   kab         rocprofv3 kernel trace of score_probe.py per build in LIBS
#               (one stream, CASES)                            -> kab_<lib>/
#   share       scripts/share_probe.py --config c3 (OPTS)       -> share.log
#   slots       bench steps in flight: SLOTS x KS, two rounds   -> slots_*.json
#   wclock      scripts/walk_clock.py --case c3 per build in LIBS -> wc_<lib>/
#   c4          scripts/c4_probe.py 29 (VARS)                   -> c4.log
#   pmc_c4      two SQ passes of C4's wide-layer replays (c4_probe.py 29
#               VARS, default 23, ULG_WALK_STATS) for c4_replay_summary.py
#   exact       scripts/probe_exact.py c3 per ULG_EXACT_PF mode in PF_MODES
#               (default "6"), two alternating rounds -> exact_<mode>_<rep>.json
# (round 5's scripts/r5_*.sh and r4_probe.sh are these steps now)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probe}
mkdir -p "$OUT"
LIBS=${LIBS:-urlearning-cpp_amd/libulg.so}
CASES=${CASES:-c3 c5}
OPTS=${OPTS:-}
FULL="python3 bench.py ${BENCH_ARGS:-}"
SHORT="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-search --no-c4 ${BENCH_ARGS:-}"
summ() {  # one line per score_probe.py case: case digest ms_median
  grep -h '"case"' "$1" | sed -E 's/.*"case": "([a-z0-9]+)".*"digest": "([0-9a-f]+)".*"ms_median": ([0-9.]+).*/\1 \2 \3/' | tr '\n' ' '
}
for step in ${STEPS:-suite smoke bench}; do
  case $step in
    suite)
      timeout -k 10 ${PYTEST_TIMEOUT:-900} python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1
      tail -n 2 "$OUT/pytest.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      tail -n 2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 400 $FULL > "$OUT/bench.json" 2> "$OUT/bench.err"
      echo "bench: $(head -c 400 "$OUT/bench.json")" ;;
    trace)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $FULL \
        > "$OUT/trace.json" 2> "$OUT/trace.log"
      echo "trace ok" ;;
    pmc_scorer)
      i=0
      for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
          "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
          "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
          "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- $SHORT \
          > "$OUT/p$i.log" 2>&1
        echo "pmc pass $i ok"
      done
      python3 scripts/pmc_r5_summarize.py "$OUT" > "$OUT/pmc_scorer.json"
      echo "pmc summary ok" ;;
    pmc_search)
      i=0
      for ctrs in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$OUT/s$i" -o run -- \
          python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c4 > "$OUT/s$i.log" 2>&1
        echo "search pmc pass $i ok"
      done
      F=$(find "$OUT/s1" -name "*counter_collection.csv" | head -1)
      W=$(find "$OUT/s2" -name "*counter_collection.csv" | head -1)
      python3 scripts/pmc_search_summarize.py "$F" "$W" c3 25 "$OUT/pmc_search_traffic.json" ;;
    probe)
      for rep in 1 2; do
        for lib in $LIBS; do
          nm=$(basename "$lib" .so)
          timeout -k 10 240 python3 scripts/score_probe.py --lib "$lib" --cases $CASES --reps 10 \
            ${OPTS:+--options $OPTS} > "$OUT/probe_${nm}_$rep.log" 2>&1
          echo "$nm rep=$rep $(summ "$OUT/probe_${nm}_$rep.log")"
        done
      done ;;
    kab)
      for lib in $LIBS; do
        nm=$(basename "$lib" .so)
        # exit 1: lists differ (timing-only probe builds); anything else ends the run
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kab_$nm" -o run -- \
          python3 scripts/score_probe.py --lib "$lib" --cases $CASES --reps 5 --options ${OPTS:-score_streams=1} \
          > "$OUT/kab_$nm.log" 2>&1 || [ $? -eq 1 ]
        echo "kab $nm: $(summ "$OUT/kab_$nm.log")"
      done ;;
    share)
      timeout -k 10 300 python3 scripts/share_probe.py --config c3 ${OPTS:+--options $OPTS} > "$OUT/share.log" 2>&1
      tail -n 1 "$OUT/share.log" | cut -c1-400 ;;
    slots)
      for rep in 1 2; do for sl in ${SLOTS:-3}; do for kk in ${KS:-2,8}; do
        ULG_SLICED_K=$kk timeout -k 10 200 python3 bench.py --steps 40 --warmup 6 --slots $sl --no-cpu-baseline \
          --no-search --no-c4 > "$OUT/slots_s${sl}_k${kk}_$rep.json" 2> "$OUT/slots_s${sl}_k${kk}_$rep.err"
        echo "slots=$sl k=$kk rep=$rep $(python3 -c "import json;d=json.load(open('$OUT/slots_s${sl}_k${kk}_$rep.json'));print(round(d['value']/1e9,3), round(d['ms_per_step'],4))")"
      done; done; done ;;
    wclock)
      for lib in $LIBS; do
        nm=$(basename "$lib" .so)
        ULG_LIB=$lib timeout -k 10 120 python3 scripts/walk_clock.py --case c3 ${OPTS:+--options $OPTS} \
          --out "$OUT/wc_$nm" > "$OUT/wclock_$nm.log" 2>&1
        echo "wclock $nm ok"
      done ;;
    c4)
      timeout -k 10 300 python3 scripts/c4_probe.py 29 ${VARS:-} > "$OUT/c4.log" 2>&1
      tail -n 3 "$OUT/c4.log" ;;
    pmc_c4)
      i=0
      for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" \
          "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"; do
        i=$((i+1))
        ULG_WALK_STATS=1 timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$OUT/c4p$i" -o run -- \
          python3 scripts/c4_probe.py 29 ${VARS:-23} > "$OUT/c4p$i.log" 2>&1
        echo "c4 pmc pass $i ok"
      done ;;
    exact)
      for rep in 1 2; do for pf in ${PF_MODES:-6}; do
        ULG_EXACT_PF=$pf timeout -k 10 240 python3 scripts/probe_exact.py c3 > "$OUT/exact_${pf}_$rep.json" 2> "$OUT/exact_${pf}_$rep.err"
        echo "exact pf=$pf rep=$rep $(cat "$OUT/exact_${pf}_$rep.json")"
      done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_probe done: ${STEPS:-suite smoke bench}"
