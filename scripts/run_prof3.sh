set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
cd /tmp && MASTER_PORT=29801 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3/graph -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof3/bench_graph.log 2>&1 || exit $?
MASTER_PORT=29802 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3/ref -- python3 $GRAFT_REPO_ROOT/bench/ref_torch_baseline.py --epochs 1 > $GRAFT_REPO_ROOT/gpurun_out/prof3/ref.log 2>&1 || exit $?
MASTER_PORT=29803 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3/pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/prof3/pmc.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python -m multidisttorch_amd.obs.stamps --json gpurun_out/prof3/stamps.json > gpurun_out/prof3/stamps.log 2>&1 && timeout -k 10 200 python -m multidisttorch_amd.obs.probe --json gpurun_out/prof3/probe.json > gpurun_out/prof3/probe.log 2>&1
