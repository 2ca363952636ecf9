#!/bin/bash
# kernel times of tile 72's two kernels (wino6_pre_k + conv_wino6_k) on the bench's tile-72 shapes
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pre72
mkdir -p $OUT
i=0
for shape in "16 38 256 512 3 1 20" "16 19 512 1024 3 1 20" "16 38 512 256 3 1 20" "16 76 128 256 3 1 20"; do
  i=$((i+1))
  MICRO_TILE=72 MICRO_RES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s$i -o s -- python tools/conv_micro.py $shape > $OUT/s$i.log 2>&1 || exit 1
  echo "== $shape"; grep -v amdgpu $OUT/s$i.log | tail -1
  python3 - "$OUT/s$i" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-40s calls %5s avg %8.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1000))
PY
done
