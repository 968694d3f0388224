set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for impl in 1 0; do
  echo "== MDT_CONV_GLDS=$impl"
  MDT_CONV_GLDS=$impl timeout -k 10 300 python bench/gemm_calib.py > gpurun_out/calib_g$impl.log 2>&1 || { tail -20 gpurun_out/calib_g$impl.log; exit 1; }
  grep -v amdgpu gpurun_out/calib_g$impl.log
done
