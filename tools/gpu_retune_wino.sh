#!/bin/bash
# Re-time the unboxed Winograd launch shapes of both committed tile caches
# (tools/retune_wino.py drops them; the bench's tuner times every applicable
# (tile, split-K) for the missing keys and writes them back), then A/B the new
# caches against the committed ones with interleaved bench runs.
#   TAGOUT=r05f [RETUNE=boxed] bash tools/gpu_retune_wino.sh
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-retune_wino}
mkdir -p $OUT
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
python tools/retune_wino.py $PKG/tiles/conv_tiles_yolov3_b16.json $OUT/yolov3_b16.json ${RETUNE:-unboxed}
python tools/retune_wino.py $PKG/tiles/conv_tiles_tiny_b256.json $OUT/tiny_b256.json ${RETUNE:-unboxed}
timeout -k 10 900 python -u bench.py --tile-cache $OUT/yolov3_b16.json --no-cpu-baseline --no-tiny > $OUT/tune_y.json 2> $OUT/tune_y.err || exit 1
timeout -k 10 900 python -u bench.py --config tiny --tile-cache $OUT/tiny_b256.json --no-cpu-baseline > $OUT/tune_t.json 2> $OUT/tune_t.err || exit 1
for rnd in 1 2; do
  for which in committed new; do
    if [ $which = committed ]; then YC=$PKG/tiles/conv_tiles_yolov3_b16.json; TC=$PKG/tiles/conv_tiles_tiny_b256.json
    else YC=$OUT/yolov3_b16.json; TC=$OUT/tiny_b256.json; fi
    timeout -k 10 300 python -u bench.py --tile-cache $YC --no-cpu-baseline --no-tiny > $OUT/y_${which}_$rnd.json 2>> $OUT/err.log || exit 1
    timeout -k 10 300 python -u bench.py --config tiny --tile-cache $TC --no-cpu-baseline > $OUT/t_${which}_$rnd.json 2>> $OUT/err.log || exit 1
    python3 -c "
import json
y=json.loads(open('$OUT/y_${which}_$rnd.json').read().strip().splitlines()[-1]); t=json.loads(open('$OUT/t_${which}_$rnd.json').read().strip().splitlines()[-1])
f=y['roofline']['families']
print('r$rnd $which yolov3', round(y['value'],1), round(y['ms_per_step'],3), 'wino', round(f.get('winograd',{}).get('ms_per_step',0),3), '| tiny', round(t['value'],1), round(t['ms_per_step'],3))" | tee -a $OUT/summary.txt
  done
done
