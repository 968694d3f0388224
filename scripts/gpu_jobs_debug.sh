# which job combinations fall back to separate launches (MDT_JOBS_DEBUG)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/jobsdbg
mkdir -p $O
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  MDT_JOBS_DEBUG=1 timeout -k 10 120 python3 bench.py --model $m --batch-size $bs --steps 2 --warmup 1 --no-graphs > $O/$m.out 2> $O/$m.err || { tail $O/$m.err; exit 1; }
  echo "== $m"; grep "\[jobs\]" $O/$m.err | sort | uniq -c || true
done
