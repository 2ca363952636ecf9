# PMC summaries of direct fp32 conv launches of the yolov3@608 B=16 step
set -e
bash tools/pmc_conv.sh gpurun_out/pmc_dA "16 608 32 64 3 2 20" 15
python3 tools/pmc_read.py gpurun_out/pmc_dA > gpurun_out/pmc_dA/summary.txt
bash tools/pmc_conv.sh gpurun_out/pmc_dB "16 76 256 128 1 1 30" 3
python3 tools/pmc_read.py gpurun_out/pmc_dB > gpurun_out/pmc_dB/summary.txt
bash tools/pmc_conv.sh gpurun_out/pmc_dC "16 152 64 128 3 1 20" 13
python3 tools/pmc_read.py gpurun_out/pmc_dC > gpurun_out/pmc_dC/summary.txt
paste gpurun_out/pmc_dA/summary.txt gpurun_out/pmc_dB/summary.txt gpurun_out/pmc_dC/summary.txt | awk '{print $1, $2, $5, $8}'
cat gpurun_out/pmc_dA/plain.txt gpurun_out/pmc_dB/plain.txt gpurun_out/pmc_dC/plain.txt
