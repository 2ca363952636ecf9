#!/bin/bash
# round 4 end state: parity numbers (-s), the default bench line, and the
# round profiles (kernel trace + FETCH/WRITE passes) of both configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04l
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_train.py -m gpu -x -v -s --timeout 500 \
    --timeout-method thread -k "tiny or windowed or yolov3_dota_608 or targeted or smoke" > "$OUT/parity.log" 2>&1
rc=$?
grep -E "patch grad|plan:|passed|failed" "$OUT/parity.log" | tail -30
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
bash tools/profile_round.sh r04 yolov3 16 fp32 && echo "prof yolov3 ok"
echo done
