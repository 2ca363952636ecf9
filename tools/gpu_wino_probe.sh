set -o pipefail
mkdir -p gpurun_out/w1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/w1/wino.log 2>&1
rc=$?
grep -E "winograd|passed|failed|Error" gpurun_out/w1/wino.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --prec fp32 --no-cpu-baseline > gpurun_out/w1/bench.json 2> gpurun_out/w1/bench.err || { tail -20 gpurun_out/w1/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/w1/bench.json').read().strip().splitlines()[-1]);print('fp32', d['value'], d['roofline']['conv_ms_per_step'], d['roofline']['frac'])"
mkdir -p gpurun_out/w1/tiles && cp adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles/*.json gpurun_out/w1/tiles/
