# PatchAdam (po_adam_amsgrad, Adam(amsgrad) + clamp in one launch) vs PyTorch's fused Adam + clamp_
# (the default; PatchAdam is opt-in: ADVPATCH_HIP_ADAM=1): the optimizer tests, then both configs' bench lines interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06adam}; mkdir -p $O
(while sleep 30; do date +%T >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_adam.py \
    "tests/test_gpu_step.py::test_two_adam_steps_yolov3" tests/test_gpu_train.py > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|PatchAdam vs|Adam step one" $O/tests.log | tail -5
for rnd in 1 2; do
  for w in torch hip; do
    if [ $w = torch ]; then E=0; else E=1; fi
    ADVPATCH_HIP_ADAM=$E timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_${w}_$rnd.json 2>> $O/err.log || exit 1
    python3 -c "
import json
d=json.loads(open('$O/b_${w}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $w yolov3', round(d['value'],1), round(d['ms_per_step'],3), '| tiny', round(d['value_tiny'],1), round(d['ms_per_step_tiny'],3))" | tee -a $O/summary.txt
  done
done
