#!/bin/bash
# MFMA counters over the bench workload's conv launches: one rocprofv3 --pmc
# pass (SQ_INSTS_MFMA, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE)
# of a short bench run, then tools/pmc_mfma_summary.py.  Usage (GPU box):
#   tools/pmc_mfma_bench.sh OUTDIR [CONFIG] [BATCH]
set -e
OUT=${1:?outdir}
CFG=${2:-yolov3}
BATCH=${3:-16}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
BENCH="bench.py --config $CFG --batch $BATCH --steps 3 --warmup 2 --no-cpu-baseline --no-tiny --prec fp32"
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex 'conv_' --output-format csv -d "$OUT/pmc" -o run -- python $BENCH \
    > "$OUT/bench_pmc.json" 2> "$OUT/pmc.err"
python tools/pmc_mfma_summary.py "$OUT" > "$OUT/mfma_summary.txt"
