# A/B of the igemm epilogue order (column-sum barrier before the global stores) using two
# prebuilt in-tree copies of _C.so (abtmp/_C_old.so, abtmp/_C_new.so); conv GPU tests on the new one
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-epi}
mkdir -p $O
cp abtmp/_C_new.so multidisttorch_amd/_C.so
timeout -k 10 400 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_conv_igemm.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/ab.txt
for rep in 1 2 3; do
  for v in old new; do
    cp abtmp/_C_$v.so multidisttorch_amd/_C.so
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv28 rep$rep $v $(python -c "import json;d=json.load(open('$O/c28.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
for rep in 1 2; do
  for v in old new; do
    cp abtmp/_C_$v.so multidisttorch_amd/_C.so
    timeout -k 10 120 python bench.py --model conv128 --batch-size 64 --steps 300 --warmup 30 > $O/c128.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv128 B=64 rep$rep $v $(python -c "import json;d=json.load(open('$O/c128.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
