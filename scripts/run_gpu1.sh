set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-graphs > gpurun_out/bench1_nographs.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench1.log; tail -2 gpurun_out/bench1_nographs.log
exit $rc
