set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench/conv_kernels.py --image 128 --batch 64 --json gpurun_out/micro128.json > gpurun_out/micro128.log 2>&1 || { tail -30 gpurun_out/micro128.log; exit 1; }
cat gpurun_out/micro128.log | grep -v amdgpu.ids
timeout -k 10 300 python bench/conv_kernels.py --image 28 --batch 128 --json gpurun_out/micro28.json > gpurun_out/micro28.log 2>&1 || { tail -30 gpurun_out/micro28.log; exit 1; }
tail -1 gpurun_out/micro28.log
