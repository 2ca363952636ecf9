# re-tune the committed conv tile cache and bench both precisions; copy the cache out
set -o pipefail
T=${1:-rt}
mkdir -p gpurun_out/$T/tiles
timeout -k 10 900 python3 -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cp adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles/*.json gpurun_out/$T/tiles/
python3 - "$T" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/%s/bench.json" % sys.argv[1]).read().strip().splitlines()[-1])
print("fp32", d["value"], d["roofline"]["conv_ms_per_step"], d["roofline"]["frac"], "| fp16x3", d.get("value_fp16x3"))
c = json.load(open("gpurun_out/%s/tiles/conv_tiles_yolov3_b16.json" % sys.argv[1]))
print("winograd launches:", sum(1 for v in c.values() if v[0] in (61, 62, 63, 64, 65, 66)), "of", len(c))
PY
