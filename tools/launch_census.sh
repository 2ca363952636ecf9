#!/bin/bash
# Steady-state launches per step of the bench workload (run on the GPU box via
# gpurun): two rocprofv3 kernel traces of the same bench command at K=5 and
# K=25 timed steps; everything outside the step loop (weights, transforms,
# tile cache, setup) cancels in the difference.  bench.py runs every timed
# step twice (plain + instrumented pass), so the difference holds 2*20 steps.
#   then, back in the build container: python tools/launch_census.py gpurun_out/census_<tag>_<cfg>
# Usage: tools/launch_census.sh TAG [CONFIG] [BATCH]
set -e
TAG=${1:?tag}
CFG=${2:-yolov3}
BATCH=${3:-16}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/census_${TAG}_${CFG}
mkdir -p "$OUT"
for K in 5 25; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/k$K" -o run -- \
      python bench.py --config "$CFG" --batch "$BATCH" --steps $K --warmup 2 --no-cpu-baseline --no-tiny \
      > "$OUT/bench_k$K.json" 2> "$OUT/k$K.err"
  echo "K=$K done"
done
