#!/bin/bash
# round 4: the full -m gpu suite (one process), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04k
mkdir -p "$OUT"
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
grep -E "patch grad|plan:|FAILED|passed|failed|Error" "$OUT/tests.log" | tail -40
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo done
