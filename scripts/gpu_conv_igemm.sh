# conv implicit-GEMM: numerics, conv-VAE benches, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -m pytest tests/gpu/test_conv_igemm.py tests/gpu/test_conv_vae_kernels.py -x -q > gpurun_out/pytest_conv.log 2>&1 || { tail -40 gpurun_out/pytest_conv.log; exit 1; }
tail -3 gpurun_out/pytest_conv.log
MASTER_PORT=29901 timeout -k 10 300 python bench.py --model conv28 --steps 200 --warmup 20 > gpurun_out/bench_conv28.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv28.log
MASTER_PORT=29902 timeout -k 10 300 python bench.py --model conv128 --batch-size 64 --steps 50 --warmup 10 > gpurun_out/bench_conv128.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv128.log
mkdir -p gpurun_out/prof_conv128 && cd /tmp && MASTER_PORT=29903 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_conv128 -- python3 $GRAFT_REPO_ROOT/bench.py --model conv128 --batch-size 64 --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_conv128/bench.log 2>&1
