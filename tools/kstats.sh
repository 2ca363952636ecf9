# Kernel time summary of a short bench run (rocprofv3 kernel trace + stats, csv).
# Usage: tools/kstats.sh OUTDIR [bench.py args...]; env passes through (e.g. PO_POOL_V1=1)
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/trace.err"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:30]:
    print("%-50s %6s %10.1f %12.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
