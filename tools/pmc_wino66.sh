# PMC passes of Winograd tiles 66 and 65 on the 152^2 64->128 yolov3 shape (tools/pmc_conv.sh)
set -e
for t in 66 65; do
  bash tools/pmc_conv.sh gpurun_out/pmc_w$t "16 152 64 128 3 1 30" $t
  python3 tools/pmc_read.py gpurun_out/pmc_w$t > gpurun_out/pmc_w$t/summary.txt
done
paste gpurun_out/pmc_w66/summary.txt gpurun_out/pmc_w65/summary.txt | awk '{print $1, $2, $5}' > gpurun_out/pmc_w66/cmp.txt
cat gpurun_out/pmc_w66/plain.txt gpurun_out/pmc_w65/plain.txt >> gpurun_out/pmc_w66/cmp.txt
