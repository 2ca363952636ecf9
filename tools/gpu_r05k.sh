#!/bin/bash
# round-5 steady-state profiles + per-launch breakdowns (yolov3 B=16, tiny B=256)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05k
timeout -k 10 300 python -u tools/step_breakdown.py --config yolov3 > gpurun_out/r05k/breakdown_yolov3.txt 2> gpurun_out/r05k/breakdown_yolov3.err
timeout -k 10 300 python -u tools/step_breakdown.py --config tiny > gpurun_out/r05k/breakdown_tiny.txt 2> gpurun_out/r05k/breakdown_tiny.err
bash tools/profile_round.sh r05 yolov3 16 fp32
bash tools/profile_round.sh r05 tiny 256 fp32
