# Round 2 first GPU pass: the driver's exact bench command (prepare-before-timing fix),
# the new conv DDP tests, then the whole GPU suite and a kernel-stats profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-r2_bench}
mkdir -p $O
export MASTER_ADDR=127.0.0.1
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$r.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
  cat $O/driver_cmd_$r.json
done
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_200_20.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_200_20.json
timeout -k 10 120 python3 bench.py --model conv128 --batch-size 64 --steps 20 --warmup 5 > $O/conv128_b64_20_5.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/conv128_b64_20_5.json
timeout -k 10 600 python -u -m pytest tests/gpu/test_conv_ddp.py -x -v --timeout 200 --timeout-method thread > $O/pytest_conv_ddp.log 2>&1 || { tail -80 $O/pytest_conv_ddp.log; exit 1; }
tail -3 $O/pytest_conv_ddp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
