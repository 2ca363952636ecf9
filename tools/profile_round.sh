#!/bin/bash
# Round profile of the bench workload (run on the GPU box via gpurun), steady
# state: every rocprofv3 pass runs the same bench command at K=5 and K=25 timed
# steps, so everything outside the step loop (weight transforms, tile cache,
# plan build, warm-up) cancels in the difference (2*20 steps: bench.py runs
# each timed step twice, plain and instrumented).
#   1. rocprofv3 --kernel-trace --stats at K=5 and K=25
#   2. FETCH_SIZE and WRITE_SIZE passes at K=5 and K=25 (they do not fit one TCC pass)
#   then, back in the build container after gpurun merged gpurun_out/:
#   python tools/pmc_summary.py gpurun_out/prof_<round>_<cfg>_<prec> <round> <cfg> <B> <prec>
#   -> profiles/<round>/summary_<cfg>_b<B>_<prec>.md + profiles/traffic_<cfg>_b<B>_<prec>.json
# Usage: tools/profile_round.sh ROUND [CONFIG] [BATCH] [PREC]
set -e
ROUND=${1:?round tag, e.g. r01}
CFG=${2:-yolov3}
BATCH=${3:-16}
PREC=${4:-fp32}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${ROUND}_${CFG}_${PREC}
mkdir -p "$OUT"
for K in 5 25; do
  BENCH="bench.py --config $CFG --batch $BATCH --steps $K --warmup 2 --no-cpu-baseline --no-tiny --prec $PREC"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_k$K" -o run -- python $BENCH \
      > "$OUT/bench_trace_k$K.json" 2> "$OUT/trace_k$K.err"
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_k$K" -o run -- python $BENCH \
      > "$OUT/bench_fetch_k$K.json" 2> "$OUT/fetch_k$K.err"
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_k$K" -o run -- python $BENCH \
      > "$OUT/bench_write_k$K.json" 2> "$OUT/write_k$K.err"
  echo "K=$K done"
done
