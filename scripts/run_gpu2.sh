set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --steps 500 --warmup 50 > gpurun_out/bench2.log 2>&1 || exit $?
tail -1 gpurun_out/bench2.log
timeout -k 10 240 python bench.py --steps 500 --warmup 50 --no-graphs > gpurun_out/bench2_ng.log 2>&1 || exit $?
tail -1 gpurun_out/bench2_ng.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/prof2/bench.log 2>&1
