#!/bin/bash
# warp phase B with the XCD-aware block remap (ADVPATCH_WARP_XCD=1, default) against blockIdx order (=0):
# bit-identity tests, FETCH_SIZE of warp_bwd_b_k, tiny-bench A/B
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-wx}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_patch_ops.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for x in 0 1; do
  ADVPATCH_WARP_XCD=$x timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'warp_bwd_b_k' --output-format csv -d $OUT/pmc_$x -o p -- python bench.py --config tiny --steps 3 --warmup 1 --no-cpu-baseline --no-tiny > $OUT/pmc_$x.log 2>&1 || { tail $OUT/pmc_$x.log; exit 1; }
  echo "xcd=$x"; python3 tools/pmc_read.py $OUT/pmc_$x | head -4
done
for rnd in 1 2; do for x in 0 1; do
  ADVPATCH_WARP_XCD=$x timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny > $OUT/tiny_${x}_$rnd.json 2> $OUT/tiny_${x}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/tiny_${x}_$rnd.json').read().strip().splitlines()[-1])
w=d['warp_roofline']
print('r$rnd xcd=$x', round(d['value'],1), round(d['ms_per_step'],3), 'bwd', round(w['po_warp_bwd']['us_per_call'],1))" | tee -a $OUT/summary.txt
done; done
