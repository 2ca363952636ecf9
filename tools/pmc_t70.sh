#!/bin/bash
# PMC of tile 70 (conv_wino5_k) on the yolov3 short-K shapes (VERDICT r3 item 4's measure)
set -e
cd "$GRAFT_REPO_ROOT"
for shape in "16 152 64 128 3 1 20" "16 76 128 256 3 1 20" "16 304 32 64 3 1 20"; do
  tag=$(echo $shape | awk '{print $2}')
  bash tools/pmc_conv.sh gpurun_out/pmc_t70_$tag "$shape" 70
  python3 tools/pmc_read.py gpurun_out/pmc_t70_$tag > gpurun_out/pmc_t70_$tag/summary.txt
  echo "== $shape"; cat gpurun_out/pmc_t70_$tag/plain.txt; grep -E "MFMA busy|per MFMA" gpurun_out/pmc_t70_$tag/summary.txt
done
