# warp pair at tiny B=256 @416: micro timings by geometry, per-kernel trace, PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06w}; mkdir -p $O
for g in ref f64 ref; do
  ADVPATCH_GEOMETRY=$g timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || { tail $O/micro.err; exit 1; }
done
cat $O/micro.txt
for g in ref f64; do
  ADVPATCH_GEOMETRY=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$g -o run -- \
    python tools/warp_bwd_micro.py > $O/tr_$g.log 2>&1 || { tail $O/tr_$g.log; exit 1; }
done
python3 -c "import glob,os,sys; print(' '.join(sorted({os.path.dirname(f) for f in glob.glob(sys.argv[1]+'/**/run_kernel_stats.csv', recursive=True)})))" $O > $O/dirs.txt
python3 tools/warp_stats.py $(cat $O/dirs.txt) | tee $O/warp_stats.txt || true
CONFIGS=tiny timeout -k 10 1000 bash tools/pmc_warp.sh || exit 1
cp -r gpurun_out/pmc_warp_tiny/summary.txt $O/pmc_warp_tiny_summary.txt
