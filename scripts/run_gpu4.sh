set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 500 python -m pytest tests/gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
MASTER_PORT=29701 timeout -k 10 600 python bench/ref_torch_baseline.py --epochs 1 > gpurun_out/ref_baseline.log 2>&1 || exit $?
tail -1 gpurun_out/ref_baseline.log
MASTER_PORT=29702 timeout -k 10 600 python bench/ref_torch_baseline.py --epochs 1 --full-epoch > gpurun_out/ref_baseline_full.log 2>&1 || exit $?
tail -1 gpurun_out/ref_baseline_full.log
mkdir -p /tmp/vh && cd /tmp/vh && MASTER_PORT=29703 timeout -k 10 600 python $GRAFT_REPO_ROOT/vae-hpo.py --ngroups 1 --epochs 3 > $GRAFT_REPO_ROOT/gpurun_out/vaehpo_e2e.log 2>&1 || exit $?
grep -E "Done|MDT_AGG|Epoch: 3 Average" $GRAFT_REPO_ROOT/gpurun_out/vaehpo_e2e.log
