set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -m pytest tests/gpu/test_e2e_gpu.py -q > gpurun_out/pytest_e2e.log 2>&1 || { tail -60 gpurun_out/pytest_e2e.log; exit 1; }
tail -2 gpurun_out/pytest_e2e.log
for m in mlp conv28 conv128; do
  B=128; [ $m = conv128 ] && B=64
  for T in 1 2; do
    MASTER_PORT=2962$T timeout -k 10 300 python bench.py --model $m --batch-size $B --trials-per-gpu $T --steps 200 --warmup 20 > gpurun_out/bench_pack_${m}_$T.log 2>&1 || { tail -20 gpurun_out/bench_pack_${m}_$T.log; exit 1; }
    tail -1 gpurun_out/bench_pack_${m}_$T.log | cut -c1-200
  done
done
