# numerics + per-launch A/B of the register-staged vs LDS-DMA conv GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/gpu/test_conv_igemm.py tests/gpu/test_conv_vae_kernels.py -x -q > gpurun_out/pytest_conv.log 2>&1 || { tail -40 gpurun_out/pytest_conv.log; exit 1; }
tail -1 gpurun_out/pytest_conv.log
for impl in 1 0; do
  MDT_CONV_GLDS=$impl timeout -k 10 300 python bench/conv_kernels.py --image 128 --batch 64 --json gpurun_out/micro128_g$impl.json > gpurun_out/micro128_g$impl.log 2>&1 || { tail -30 gpurun_out/micro128_g$impl.log; exit 1; }
done
paste <(awk '{print $1, $2, $3, $4}' gpurun_out/micro128_g1.log) <(awk '{print $4}' gpurun_out/micro128_g0.log) | grep -v amdgpu
