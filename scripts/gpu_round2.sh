# conv + rccl numerics, conv microbench and benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -m pytest tests/gpu/test_conv_igemm.py tests/gpu/test_conv_vae_kernels.py tests/gpu/test_rccl_reducer.py -x -q > gpurun_out/pytest_r2.log 2>&1 || { tail -40 gpurun_out/pytest_r2.log; exit 1; }
tail -2 gpurun_out/pytest_r2.log
timeout -k 10 300 python bench/conv_kernels.py --image 128 --batch 64 --json gpurun_out/micro128.json > gpurun_out/micro128.log 2>&1 || { tail -30 gpurun_out/micro128.log; exit 1; }
grep -v amdgpu.ids gpurun_out/micro128.log
MASTER_PORT=29901 timeout -k 10 300 python bench.py --model conv28 --steps 200 --warmup 20 > gpurun_out/bench_conv28.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv28.log
MASTER_PORT=29902 timeout -k 10 300 python bench.py --model conv128 --batch-size 64 --steps 50 --warmup 10 > gpurun_out/bench_conv128.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv128.log
