#!/bin/bash
# PMC of the direct 1x1 launches of the yolov3 step (tile 11, 76^2 256->128; tile 9, 304^2 64->32)
set -e
cd "$GRAFT_REPO_ROOT"
for spec in "16 76 256 128 1 1 30:11" "16 304 64 32 1 1 20:9" "16 608 32 64 3 2 20:16"; do
  shape=${spec%%:*}; tile=${spec##*:}
  tag=$(echo $shape | awk '{print $2"_"$3"_"$5}')
  bash tools/pmc_conv.sh gpurun_out/pmc_d_$tag "$shape" $tile
  python3 tools/pmc_read.py gpurun_out/pmc_d_$tag > gpurun_out/pmc_d_$tag/summary.txt
  echo "== $shape tile $tile"; cat gpurun_out/pmc_d_$tag/plain.txt
  grep -E "MFMA busy|per MFMA|SQ_WAIT_INST_ANY|SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_ACTIVE_INST_ANY|SQ_INST_LEVEL_VMEM|SQ_WAVES " gpurun_out/pmc_d_$tag/summary.txt
done
