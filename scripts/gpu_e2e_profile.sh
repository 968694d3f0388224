set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e && cd gpurun_out/e2e
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29631
timeout -k 10 600 python $GRAFT_REPO_ROOT/vae-hpo.py --ngroups 1 --epochs 3 --profile --metrics-dir m > run.log 2>&1 || { tail -30 run.log; exit 1; }
grep -E "MDT_AGGREGATE|Done" run.log
cat m/trial-0.jsonl
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/gpu/test_e2e_gpu.py -q > gpurun_out/pytest_e2e.log 2>&1 || { tail -40 gpurun_out/pytest_e2e.log; exit 1; }
tail -1 gpurun_out/pytest_e2e.log
