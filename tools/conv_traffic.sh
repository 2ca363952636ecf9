#!/bin/bash
# Per-launch conv time and HBM traffic of the bench step (GPU box):
#   kernel trace + FETCH_SIZE pass + WRITE_SIZE pass over tools/step_breakdown.py
# then (here or there): python tools/conv_traffic.py OUTDIR
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/conv_traffic}
CFG=${2:-yolov3}
BATCH=${3:-$([ "$CFG" = tiny ] && echo 256 || echo 16)}
mkdir -p "$OUT"
ARGS="tools/step_breakdown.py --config $CFG --batch $BATCH --steps 3"
export ADVPATCH_TUNE_CACHE=$GRAFT_REPO_ROOT/adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles/conv_tiles_${CFG}_b${BATCH}.json
BREAKDOWN_JSON=$OUT/launches.json timeout -k 10 300 python $ARGS > "$OUT/breakdown.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python $ARGS > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python $ARGS > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python $ARGS > "$OUT/write.log" 2>&1
