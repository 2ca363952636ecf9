set -e
python3 - <<'PY'
import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    try: print(p, open(p).read().strip())
    except Exception as e: print(p, e)
PY
ADVPATCH_CONV_PREC=fp32 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/diag1_bench_fp32.json 2> gpurun_out/diag1_bench_fp32.err
cat gpurun_out/diag1_bench_fp32.json
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "yolov3_dota_608" > gpurun_out/diag1_step.log 2>&1
grep -E "vs float64|passed|failed" gpurun_out/diag1_step.log
