# full GPU suite + bench (3 models) + conv timelines after the finalize/Adam vectorisation
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 180 python3 bench.py > $O/bench_conv28.json 2> $O/bench_conv28.err || { tail $O/bench_conv28.err; exit 1; }
timeout -k 10 180 python3 bench.py --model conv128 --batch-size 64 > $O/bench_conv128.json 2> $O/bench_conv128.err || exit 1
timeout -k 10 180 python3 bench.py --model mlp > $O/bench_mlp.json 2> $O/bench_mlp.err || exit 1
cat $O/bench_*.json
OUT=$GRAFT_REPO_ROOT/$O/tl
mkdir -p $OUT
cd /tmp
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$m -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --model $m --batch-size $bs --steps 40 --warmup 10 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  f=$(find $OUT/$m -name '*kernel_trace.csv' | head -1)
  python3 $GRAFT_REPO_ROOT/scripts/ktimeline.py $f "thin_conv_k<32, 4, float>" 10 > $OUT/${m}_timeline.txt
  tail -4 $OUT/${m}_timeline.txt
  rm -f $f
done
