set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m multidisttorch_amd.obs.stamps --json gpurun_out/stamps.json > gpurun_out/stamps.log 2>&1 || exit $?
python multidisttorch_amd/obs/show_stamps.py
timeout -k 10 240 python bench.py --steps 500 --warmup 50 > gpurun_out/bench3.log 2>&1 || exit $?
tail -1 gpurun_out/bench3.log
