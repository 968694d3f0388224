set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
MASTER_PORT=29901 timeout -k 10 300 python bench.py --model conv28 --steps 200 --warmup 20 > gpurun_out/bench_conv28.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv28.log
MASTER_PORT=29902 timeout -k 10 300 python bench.py --model conv128 --batch-size 64 --steps 50 --warmup 10 > gpurun_out/bench_conv128.log 2>&1 || exit $?
tail -1 gpurun_out/bench_conv128.log
mkdir -p gpurun_out/prof_conv && cd /tmp && MASTER_PORT=29903 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_conv -- python3 $GRAFT_REPO_ROOT/bench.py --model conv28 --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_conv/bench.log 2>&1
