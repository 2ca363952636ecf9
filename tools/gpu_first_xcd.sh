#!/bin/bash
# first-layer kernels with the XCD-aware block remap (ADVPATCH_FIRST_XCD=1, default) against blockIdx order (=0):
# tests, FETCH_SIZE per dispatch, bench A/B (yolov3 line + tiny line)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-fx}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_first_conv.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for x in 0 1; do
  ADVPATCH_FIRST_XCD=$x timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'first_' --output-format csv -d $OUT/pmc_$x -o p -- python tools/first_micro.py 5 > $OUT/pmc_$x.log 2>&1 || { tail $OUT/pmc_$x.log; exit 1; }
done
for rnd in 1 2; do for x in 0 1; do
  ADVPATCH_FIRST_XCD=$x timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/b_${x}_$rnd.json 2> $OUT/b_${x}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${x}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd xcd=$x', round(d['value'],1), round(d['ms_per_step'],3), 'first', round(d['warp_roofline']['first_layer']['us_per_call'],1), '| tiny', round(d['value_tiny'],1), round(d['ms_per_step_tiny'],3), 'first', round(d['warp_roofline_tiny']['first_layer']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
