#!/bin/bash
# One GPU call: bench (writes the conv tile cache), copy the cache out, then the -m gpu suite.
# Usage: tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
mkdir -p gpurun_out/$TAG
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
timeout -k 10 600 python3 -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 3000 gpurun_out/$TAG/bench.json
mkdir -p gpurun_out/$TAG/tiles && cp $PKG/tiles/*.json gpurun_out/$TAG/tiles/ 2>/dev/null
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread "${KA[@]}" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
grep -E "vs float64|passed|failed|Error|error" gpurun_out/$TAG/pytest.log | tail -40
exit $rc
