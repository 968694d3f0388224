# MFMA VGPR-form build: direct-kernel numerics + stamps, conv128 per-launch + bench, conv tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-vgprform}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/gpu/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dconv.log 2>&1 || { tail -40 $O/pytest_dconv.log; exit 1; }
tail -1 $O/pytest_dconv.log
timeout -k 10 120 python bench/dconv_stamps.py --json $O/stamps.json > $O/stamps.txt 2>&1 || { tail -30 $O/stamps.txt; exit 1; }
grep -v amdgpu $O/stamps.txt
timeout -k 10 180 python bench/conv_kernels.py --image 128 --batch 64 --reps 20 --json $O/per_launch.json > $O/per_launch.txt 2>&1 || { tail -30 $O/per_launch.txt; exit 1; }
grep -E "^ +[0-9]+ (igemm|thin|launch_jobs|combine|reparam|grad_fin|wtrans)" $O/per_launch.txt | grep -v " 1\.[0-9][0-9] us\| 0\.[0-9][0-9] us" | cut -c1-60
for b in 64 128; do
timeout -k 10 180 python3 bench.py --model conv128 --batch-size $b --steps 50 --warmup 10 > $O/bench_c128_$b.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c128_$b.json'));print('conv128 B=$b', d['ms_per_step'], 'ms', d['value'])"
done
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_c28.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c28.json'));print('conv28', d['ms_per_step'], 'ms', d['value'])"
timeout -k 10 400 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_conv_ddp.py -q --timeout 150 --timeout-method thread > $O/pytest_conv.log 2>&1 || { tail -40 $O/pytest_conv.log; exit 1; }
tail -2 $O/pytest_conv.log
