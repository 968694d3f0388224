# Round-1 state check: GPU suite, smoke(), default bench (the driver's command), kernel stats of it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 180 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 180 python bench.py --model conv128 --batch-size 64 > $O/bench_conv128.json 2> $O/bench_conv128.err || { tail -20 $O/bench_conv128.err; exit 1; }
cat $O/bench_conv128.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
