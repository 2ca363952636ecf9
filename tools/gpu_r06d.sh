set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u tools/sqrt_probe.py gpurun_out/r06d > gpurun_out/r06d/sqrt_probe.txt 2>&1
true
