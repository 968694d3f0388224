set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench/packing.py --model mlp > gpurun_out/packing_q$q.log 2>&1 || { tail -20 gpurun_out/packing_q$q.log; exit 1; }
  grep '^{' gpurun_out/packing_q$q.log
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench/packing.py --model conv28 --trials 1,2,4 > gpurun_out/packing_c28_q$q.log 2>&1 || { tail -20 gpurun_out/packing_c28_q$q.log; exit 1; }
  grep '^{' gpurun_out/packing_c28_q$q.log
done
