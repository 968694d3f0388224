# Fused 28x28 step: per-launch timing + LDS bank-conflict counters
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-f28parts}
mkdir -p $O
timeout -k 10 120 python bench/f28_parts.py --json $O/parts.json > $O/parts.txt 2>&1 || { tail -30 $O/parts.txt; exit 1; }
grep -v amdgpu.ids $O/parts.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-graphs > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/pmc.log; exit 1; }
echo pmc done
