# A/B of the phase-B gather (warp_bwd_b_k): this tree vs the round-5 tree
# (_ab_r05, a detached worktree of 5e105a4), PMC passes on tiny B=256 @416.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
for t in cur r05; do
  if [ $t = r05 ]; then D=_ab_r05; else D=.; fi
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_COUNT"; do
    i=$((i+1))
    (cd $D && ADVPATCH_GEOMETRY=f64 timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex 'warp_bwd_b' --output-format csv \
       -d $GRAFT_REPO_ROOT/$O/$t/p$i -o p$i -- python bench.py --config tiny --steps 3 --warmup 2 --no-cpu-baseline --no-tiny \
       > $GRAFT_REPO_ROOT/$O/$t.p$i.log 2>&1) || { echo "pass $t $i failed"; tail $O/$t.p$i.log; exit 1; }
  done
  echo "== $t"; PMC_BY_KERNEL=1 python3 tools/pmc_read.py $O/$t | tee $O/$t.summary.txt
done
