#!/bin/bash
# first-layer output stores non-temporal (ADVPATCH_FIRST_NT=1) vs plain (=0, default)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-fnt}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_first_conv.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
ADVPATCH_FIRST_NT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_first_conv.py -x -q --timeout 120 --timeout-method thread >> $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
grep passed $OUT/tests.txt
for rnd in 1 2; do for x in 0 1; do
  ADVPATCH_FIRST_NT=$x timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/b_${x}_$rnd.json 2> $OUT/b_${x}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${x}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd nt=$x', round(d['value'],1), round(d['ms_per_step'],3), 'first', round(d['warp_roofline']['first_layer']['us_per_call'],1), '| tiny', round(d['value_tiny'],1), round(d['ms_per_step_tiny'],3), 'first', round(d['warp_roofline_tiny']['first_layer']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
