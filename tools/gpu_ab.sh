#!/bin/bash
# Interleaved A/B bench runs of the default line against the same line with an
# environment override (e.g. AB_ENV="ADVPATCH_TILE_MAP=68:70").
# Usage (on the box): AB_ENV="VAR=value ..." tools/gpu_ab.sh TAG [ROUNDS] [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:?tag}; shift
ROUNDS=${1:-2}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for which in A B; do
    if [ $which = A ]; then E=""; else E="$AB_ENV"; fi
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/${which}_$r.json" 2>> "$OUT/err.log" || { echo "bench $which failed"; tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/${which}_$r.json').read().strip().splitlines()[-1])
print('r$r $which', round(d['value'],1), round(d['ms_per_step'],3), 'conv', round(d['roofline']['conv_ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), '| tiny', round(d.get('value_tiny',0),1), round(d.get('ms_per_step_tiny',0),3))" | tee -a "$OUT/summary.txt"
  done
done
