#!/bin/bash
# boxed-launch probe -> per-key best choices in a new cache (gpurun_out/bp/<cfg>_new.json), then a
# step-level A/B of the committed cache against it
cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-yolov3}; B=${B:-16}
OUT=gpurun_out/bp
mkdir -p $OUT
OLD=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles/conv_tiles_${CFG}_b${B}.json
PROBE_WRITE=$OUT/${CFG}_new.json PROBE_WINO_ON_DIRECT=1 timeout -k 10 600 python -u tools/boxed_probe.py $CFG 20 > $OUT/${CFG}_apply.txt 2>&1 || { tail $OUT/${CFG}_apply.txt; exit 1; }
grep "^key\|updated\|boxed launches" $OUT/${CFG}_apply.txt | cut -c1-220
NOTINY=""; [ $CFG = yolov3 ] && NOTINY="--no-tiny"
for rnd in 1 2 3; do for c in old new; do
  TC=$OLD; [ $c = new ] && TC=$OUT/${CFG}_new.json
  timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline $NOTINY --no-tiny --tile-cache $TC > $OUT/ab_${CFG}_${c}_$rnd.json 2> $OUT/ab_${CFG}_${c}_$rnd.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${CFG}_${c}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $c', round(d['value'],1), round(d['ms_per_step'],3), 'conv', round(d['roofline']['conv_ms_per_step'],3))" | tee -a $OUT/ab_${CFG}_summary.txt
done; done
