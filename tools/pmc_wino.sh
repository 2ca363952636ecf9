set -e
bash tools/pmc_conv.sh gpurun_out/pmc_w62 "16 38 512 256 3 1 30" 62
python3 tools/pmc_read.py gpurun_out/pmc_w62 > gpurun_out/pmc_w62/summary.txt
bash tools/pmc_conv.sh gpurun_out/pmc_d11 "16 38 512 256 3 1 30" 4
python3 tools/pmc_read.py gpurun_out/pmc_d11 > gpurun_out/pmc_d11/summary.txt
paste gpurun_out/pmc_w62/summary.txt gpurun_out/pmc_d11/summary.txt | awk '{print $1, $2, $5}'
cat gpurun_out/pmc_w62/plain.txt gpurun_out/pmc_d11/plain.txt
