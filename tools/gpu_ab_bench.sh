#!/bin/bash
# A/B bench of ablation libraries (tools/abl/libadvpatch_<TAG>.so; "base" = the in-tree build):
#   LIBS="base ntw" ROUNDS=2 TAGOUT=r03x bash tools/gpu_ab_bench.sh
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-ab}
mkdir -p $OUT
for rnd in $(seq ${ROUNDS:-2}); do
for lib in ${LIBS:-base}; do
  L=""; [ $lib != base ] && L=${ABLDIR:-tools/abl}/libadvpatch_$lib.so
  ADVPATCH_LIB=$L timeout -k 10 400 python -u bench.py --prec fp32 --no-cpu-baseline > $OUT/bench_${lib}_$rnd.json 2> $OUT/bench_${lib}_$rnd.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('$OUT/bench_${lib}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $lib', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['conv_ms_per_step'],3), 'direct', round(d['roofline']['families']['direct']['ms_per_step'],3), '| tiny', round(d.get('value_tiny',0),1), round(d.get('ms_per_step_tiny',0),3))" | tee -a $OUT/summary.txt
done; done
