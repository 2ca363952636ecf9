#!/bin/bash
# Round profile of the bench workload (run on the GPU box via gpurun):
#   1. one plain bench run (writes the synthetic weights and the conv tile cache)
#   2. rocprofv3 --kernel-trace --stats of the same bench command
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass)
#   then, back in the build container after gpurun merged gpurun_out/:
#   python tools/pmc_summary.py gpurun_out/prof_<round>_<cfg> <round> <cfg> <B> 22
#   -> profiles/<round>/ + profiles/traffic_<cfg>_b<B>.json
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
STEPS=10
WARM=2
BENCH="bench.py --config $CFG --batch $BATCH --steps $STEPS --warmup $WARM --no-cpu-baseline --no-tiny --prec $PREC"
timeout -k 10 300 python $BENCH > "$OUT/bench_plain.json" 2> "$OUT/bench_plain.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python $BENCH \
    > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python $BENCH \
    > "$OUT/bench_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python $BENCH \
    > "$OUT/bench_write.json" 2> "$OUT/pmc_write.err"
ADVPATCH_CONV_PREC=$PREC tools/conv_traffic.sh "$OUT/conv_traffic" "$CFG" "$BATCH" > "$OUT/conv_traffic.log" 2>&1
python tools/pmc_summary.py "$OUT" "$ROUND" "$CFG" "$BATCH" $((2 * STEPS + WARM)) "$PREC" > "$OUT/summary.txt"
python tools/conv_traffic.py "$OUT/conv_traffic" --top 60 > "$OUT/conv_traffic.txt"
