set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1/a -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/pmc1/a.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1/b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/pmc1/b.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1/c -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/pmc1/c.log 2>&1
