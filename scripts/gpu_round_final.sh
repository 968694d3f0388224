# End-of-session validation of the committed tree: GPU suite, smoke, benches, N=2 launch rehearsal, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final2
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for r in 1 2; do
  timeout -k 10 120 python bench.py > $O/bench_default_$r.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
  cat $O/bench_default_$r.json
done
timeout -k 10 120 python bench.py --model conv128 --batch-size 64 > $O/bench_conv128_b64.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_conv128_b64.json
timeout -k 10 120 python bench.py --model conv128 > $O/bench_conv128_b128.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_conv128_b128.json
timeout -k 10 120 python bench.py --model mlp > $O/bench_mlp.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_mlp.json
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29951 bench.py --gpus 2 --steps 100 --warmup 10 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
