# A/B of the register-staged k-loop barrier / prefetch depth, four prebuilt in-tree _C.so
# variants (abtmp/_C_v{0..3}.so): v0 __syncthreads PF=1 (default), v1 s_barrier PF=1,
# v2 s_barrier PF=2, v3 s_barrier PF=auto(3/2). Conv GPU tests on each variant first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/kbar
mkdir -p $O
for v in 1 2 3; do
  cp abtmp/_C_v$v.so multidisttorch_amd/_C.so
  timeout -k 10 300 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_conv_igemm.py -x -q --timeout 120 --timeout-method thread > $O/pytest_v$v.log 2>&1 || { tail -40 $O/pytest_v$v.log; exit 1; }
  echo "v$v $(tail -1 $O/pytest_v$v.log)"
done
: > $O/ab.txt
for rep in 1 2; do
  for v in 0 1 2 3; do
    cp abtmp/_C_v$v.so multidisttorch_amd/_C.so
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv28 rep$rep v$v $(python -c "import json;d=json.load(open('$O/c28.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
    timeout -k 10 120 python bench.py --model conv128 --batch-size 64 --steps 300 --warmup 30 > $O/c128.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv128 B=64 rep$rep v$v $(python -c "import json;d=json.load(open('$O/c128.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
cp abtmp/_C_v0.so multidisttorch_amd/_C.so
