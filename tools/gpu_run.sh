#!/bin/bash
# One GPU call of a round: selected -m gpu tests, the default bench line, and
# (optionally) the 2-rank gloo rehearsal of bench.py --gpus 2.
# Usage (on the box, via gpurun): tools/gpu_run.sh TAG [PYTEST_K|all|none] [bench|nobench] [gloo]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:?tag}
K=${2:-none}
B=${3:-bench}
G=${4:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$K" != "none" ]; then
  if [ "$K" = "all" ]; then KA=(); else KA=(-k "$K"); fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread "${KA[@]}" \
      > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "patch grad|plan:|PASSED|FAILED|passed|failed|Error" "$OUT/tests.log" | tail -60
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if [ "$B" = "bench" ]; then
  timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
  cut -c1-600 "$OUT/bench.json"
fi
if [ "$G" = "gloo" ]; then
  timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 \
      > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err" || { echo "gloo rc=$?"; tail -20 "$OUT/bench_gloo2.err"; exit 1; }
  cut -c1-400 "$OUT/bench_gloo2.json"
fi
echo done
