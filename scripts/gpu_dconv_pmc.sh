set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-dconv_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/p1 -o p1 -- python3 $GRAFT_REPO_ROOT/bench/dconv_stamps.py --reps 3 > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/p2 -o p2 -- python3 $GRAFT_REPO_ROOT/bench/dconv_stamps.py --reps 3 > $GRAFT_REPO_ROOT/$O/p2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/p2.log; exit 1; }
echo done
