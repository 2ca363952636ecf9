set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 300 python tools/affine_grid_probe.py > gpurun_out/r06b/affine_probe.txt 2>&1
timeout -k 10 300 python -m pytest -q tests/test_geometry_ref.py -k "grid_sample or linspace or theta or sin_cos or fma" -p no:cacheprovider > gpurun_out/r06b/geom_cpu_tests.txt 2>&1
lscpu > gpurun_out/r06b/lscpu.txt 2>&1
python -c "import torch; print(torch.__config__.show())" > gpurun_out/r06b/torch_config.txt 2>&1
true
