# full GPU validation: all gpu tests, smoke, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
MASTER_PORT=29911 timeout -k 10 300 python bench.py > gpurun_out/bench_mlp.log 2>&1 || { tail -20 gpurun_out/bench_mlp.log; exit 1; }
tail -1 gpurun_out/bench_mlp.log
