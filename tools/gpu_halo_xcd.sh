#!/bin/bash
# tile 69 (conv_halo_pool_k) with the XCD-aware tile walk (ADVPATCH_HALO_XCD=1, default) vs blockIdx order (=0)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-hx}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for x in 0 1; do
  ADVPATCH_HALO_XCD=$x timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'conv_halo' --output-format csv -d $OUT/pmc_$x -o p -- python bench.py --config tiny --steps 3 --warmup 1 --no-cpu-baseline --no-tiny > $OUT/pmc_$x.log 2>&1 || { tail $OUT/pmc_$x.log; exit 1; }
done
for rnd in 1 2; do for x in 0 1; do
  ADVPATCH_HALO_XCD=$x timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny > $OUT/tiny_${x}_$rnd.json 2> $OUT/tiny_${x}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/tiny_${x}_$rnd.json').read().strip().splitlines()[-1])
f=d['roofline']['families'].get('halo',{})
print('r$rnd xcd=$x', round(d['value'],1), round(d['ms_per_step'],3), 'halo ms', round(f.get('ms_per_step',0),3))" | tee -a $OUT/summary.txt
done; done
