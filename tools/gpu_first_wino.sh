#!/bin/bash
# First-layer F(2x2) form: parity tests, micro timing, tiny-bench A/B (ADVPATCH_FIRST_WINO=0/1)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-fw}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_first_conv.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 120 python -u tools/first_micro.py 50 > $OUT/micro.txt 2>&1 || { cat $OUT/micro.txt; exit 1; }
cat $OUT/micro.txt
for rnd in 1 2; do for fw in 0 1; do
  ADVPATCH_FIRST_WINO=$fw timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny > $OUT/tiny_${fw}_$rnd.json 2> $OUT/tiny_${fw}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/tiny_${fw}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd wino=$fw', round(d['value'],1), round(d['ms_per_step'],3), round(d['warp_roofline']['first_layer']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
