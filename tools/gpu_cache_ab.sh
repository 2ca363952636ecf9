#!/bin/bash
# tiny bench A/B of two tile caches: tools/abl_now/tiny_old.json vs the committed one
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-cab}
mkdir -p $OUT
NEW=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles/conv_tiles_tiny_b256.json
for rnd in 1 2 3; do for c in old new; do
  TC=tools/abl_now/tiny_old.json; [ $c = new ] && TC=$NEW
  timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline --no-tiny --tile-cache $TC > $OUT/t_${c}_$rnd.json 2> $OUT/t_${c}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/t_${c}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $c', round(d['value'],1), round(d['ms_per_step'],3), 'direct', round(d['roofline']['families']['direct']['ms_per_step'],3))" | tee -a $OUT/summary.txt
done; done
