# per-launch timeline of one conv28 / conv128 step (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/tl2
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$m -o trace -- python3 $R/bench.py --model $m --batch-size $bs --steps 40 --warmup 10 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  f=$(find $OUT/$m -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/ktimeline.py $f "thin_conv_k<32, 4, float>" 10 > $OUT/${m}_timeline.txt
  cat $OUT/${m}_timeline.txt
  rm -f $f
done
