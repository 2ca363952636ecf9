#!/bin/bash
# Forward-saved warp factors (ADVPATCH_WARP_FAC=1, default) against the re-evaluating backward (=0):
# bit-identity tests, tiny-bench A/B
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-wf}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_patch_ops.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for rnd in 1 2; do for wf in 0 1; do
  ADVPATCH_WARP_FAC=$wf timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny > $OUT/tiny_${wf}_$rnd.json 2> $OUT/tiny_${wf}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/tiny_${wf}_$rnd.json').read().strip().splitlines()[-1])
w=d['warp_roofline']
print('r$rnd fac=$wf', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(w['po_warp_fwd']['us_per_call'],1), 'bwd', round(w['po_warp_bwd']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
