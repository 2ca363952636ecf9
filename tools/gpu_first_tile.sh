#!/bin/bash
# First layer: LDS-tiled pooled kernel (ADVPATCH_FIRST_TILE=1, default) against the per-pixel gathers (=0):
# parity tests, micro timing, tiny-bench A/B
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-ft}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_first_conv.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for lt in 0 1; do
  ADVPATCH_FIRST_TILE=$lt timeout -k 10 120 python -u tools/first_micro.py 50 > $OUT/micro_$lt.txt 2>&1 || { cat $OUT/micro_$lt.txt; exit 1; }
  echo "tile=$lt"; grep pool $OUT/micro_$lt.txt
done
for rnd in 1 2; do for lt in 0 1; do
  ADVPATCH_FIRST_TILE=$lt timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny > $OUT/tiny_${lt}_$rnd.json 2> $OUT/tiny_${lt}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/tiny_${lt}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd tile=$lt', round(d['value'],1), round(d['ms_per_step'],3), round(d['warp_roofline']['first_layer']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
