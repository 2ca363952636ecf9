# round-6 steady-state profile of one config (tools/profile_round.sh) + its per-launch breakdown
# usage: tools/gpu_r06prof.sh yolov3 16 | tiny 256
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${1:?config}; B=${2:?batch}
mkdir -p gpurun_out/r06prof
timeout -k 10 1000 bash tools/profile_round.sh r06 $CFG $B fp32 || { echo "profile failed"; exit 1; }
timeout -k 10 300 python -u tools/step_breakdown.py --config $CFG --steps 5 > gpurun_out/r06prof/step_breakdown_${CFG}_b$B.txt 2>&1 || exit 1
tail -2 gpurun_out/r06prof/step_breakdown_${CFG}_b$B.txt
