#!/bin/bash
# End-of-round GPU checks (run via gpurun):
#   suite   - the whole -m gpu suite in one process
#   parity  - the step parity tests with their printed errors (-s)
#   bench   - the default bench line
#   profile - tools/profile_round.sh of both configs
# Usage: tools/gpu_round_end.sh ROUND STAGE...   e.g.  tools/gpu_round_end.sh r04 parity bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROUND=${1:?round tag}
shift
OUT=gpurun_out/$ROUND
mkdir -p "$OUT"
for stage in "$@"; do
  case $stage in
    suite)
      # heartbeat: a test that runs for minutes writes nothing to suite.log until it ends
      (while sleep 30; do date +%T >> "$OUT/heartbeat"; done) & HB=$!
      timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
          > "$OUT/suite.log" 2>&1
      rc=$?
      kill $HB
      [ $rc -eq 0 ] || { echo "suite failed"; grep -E "FAILED|Error" "$OUT/suite.log" | tail -20; exit 1; }
      tail -1 "$OUT/suite.log" ;;
    parity)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_train.py -m gpu -x -v -s \
          --timeout 500 --timeout-method thread -k "tiny or windowed or yolov3_dota_608 or targeted" \
          > "$OUT/parity.log" 2>&1 || { echo "parity failed"; tail -30 "$OUT/parity.log"; exit 1; }
      grep -E "patch grad|plan:|passed" "$OUT/parity.log" | tail -20 ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
          || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
      cut -c1-300 "$OUT/bench.json" ;;
    profile)
      bash tools/profile_round.sh "$ROUND" yolov3 16 fp32 && bash tools/profile_round.sh "$ROUND" tiny 256 fp32 \
          || { echo "profile failed"; exit 1; }
      echo "profiles in gpurun_out/prof_${ROUND}_*" ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo done
