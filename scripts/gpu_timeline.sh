# in-graph kernel timeline of one training step (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/tl
mkdir -p $OUT
for m in ${MODELS:-conv28}; do
  bs=128; [ $m = conv128 ] && bs=64
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$m -o trace -- python3 bench.py --model $m --batch-size $bs --steps 40 --warmup 10 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  f=$(find $OUT/$m -name '*kernel_trace.csv' | head -1)
  python3 scripts/ktimeline.py $f "${MARK:-thin_conv_k<32, 4, float>}" 10 > $OUT/${m}_timeline.txt
  cat $OUT/${m}_timeline.txt
  rm -f $f
done
