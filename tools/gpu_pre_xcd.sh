#!/bin/bash
# wino6_pre_k in XCD-aware block order (ADVPATCH_PRE_XCD=1, default) vs launch order (=0)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-px}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wino6.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for x in 0 1; do
  ADVPATCH_PRE_XCD=$x timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'wino6_pre_k' --output-format csv -d $OUT/pmc_$x -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-tiny > $OUT/pmc_$x.log 2>&1 || { tail $OUT/pmc_$x.log; exit 1; }
done
for rnd in 1 2; do for x in 0 1; do
  ADVPATCH_PRE_XCD=$x timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/b_${x}_$rnd.json 2> $OUT/b_${x}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/b_${x}_$rnd.json').read().strip().splitlines()[-1])
f=d['roofline']['families']['winograd']
print('r$rnd xcd=$x', round(d['value'],1), round(d['ms_per_step'],3), 'wino ms', round(f['ms_per_step'],3), '| tiny', round(d['value_tiny'],1), round(d['ms_per_step_tiny'],3))" | tee -a $OUT/summary.txt
done; done
