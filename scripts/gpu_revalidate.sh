# Re-validation after a rebuild: GPU tests, smoke, the three bench models, a kernel-stats profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reval
O=gpurun_out/reval
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
MASTER_PORT=29911 timeout -k 10 300 python bench.py > $O/bench_default.json 2>$O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
MASTER_PORT=29912 timeout -k 10 300 python bench.py --model conv128 > $O/bench_conv128.json 2>$O/bench_conv128.err || { tail -20 $O/bench_conv128.err; exit 1; }
cat $O/bench_conv128.json
MASTER_PORT=29913 timeout -k 10 300 python bench.py --model mlp > $O/bench_mlp.json 2>$O/bench_mlp.err || { tail -20 $O/bench_mlp.err; exit 1; }
cat $O/bench_mlp.json
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=29914 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
