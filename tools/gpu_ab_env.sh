#!/bin/bash
# Interleaved A/B of environment settings on the bench (yolov3 + tiny lines):
#   AB="base|ADVPATCH_TILE_MAP=70:71" ROUNDS=2 TAGOUT=r05d bash tools/gpu_ab_env.sh
# ("base" = no extra setting; settings separated by '|', several in one arm by ',')
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-abenv}
mkdir -p $OUT
IFS='|' read -ra ARMS <<< "${AB:-base}"
for rnd in $(seq ${ROUNDS:-2}); do
  i=0
  for arm in "${ARMS[@]}"; do
    i=$((i+1))
    envs=()
    [ "$arm" != base ] && IFS=',' read -ra envs <<< "$arm"
    env "${envs[@]}" timeout -k 10 400 python -u bench.py --prec fp32 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench_${i}_$rnd.json 2> $OUT/bench_${i}_$rnd.err || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/bench_${i}_$rnd.json').read().strip().splitlines()[-1]); r=d['roofline']; f=r['families']
print('r$rnd [$arm]', round(d['value'],1), round(d['ms_per_step'],3), 'conv', round(r['conv_ms_per_step'],3), 'wino', round(f.get('winograd',{}).get('ms_per_step',0),3), 'direct', round(f['direct']['ms_per_step'],3), '| tiny', round(d.get('value_tiny',0),1), round(d.get('ms_per_step_tiny',0),3))" | tee -a $OUT/summary.txt
  done
done
