# torch-eager anchors for the conv-VAE (reference loop, bf16 autocast) + per-launch conv28 breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/anchor
timeout -k 10 300 python bench/ref_torch_baseline.py --model conv28 > gpurun_out/anchor/ref_conv28.json 2> gpurun_out/anchor/ref_conv28.err
timeout -k 10 300 python bench/ref_torch_baseline.py --model conv128 --batch-size 64 > gpurun_out/anchor/ref_conv128.json 2> gpurun_out/anchor/ref_conv128.err
timeout -k 10 300 python bench/ref_torch_baseline.py > gpurun_out/anchor/ref_mlp.json 2> gpurun_out/anchor/ref_mlp.err
timeout -k 10 300 python bench/conv_kernels.py --image 28 --batch 128 --json gpurun_out/anchor/micro28.json > gpurun_out/anchor/micro28.log 2>&1
cat gpurun_out/anchor/*.json | grep what
grep -v amdgpu.ids gpurun_out/anchor/micro28.log
