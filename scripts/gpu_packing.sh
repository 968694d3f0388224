set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in mlp conv28 conv128; do
  timeout -k 10 300 python bench/packing.py --model $m > gpurun_out/packing_$m.log 2>&1 || { tail -20 gpurun_out/packing_$m.log; exit 1; }
  grep '^{' gpurun_out/packing_$m.log
done
