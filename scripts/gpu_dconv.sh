# direct conv kernels: numerics, per-launch A/B vs the im2col kernels, conv128 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-dconv}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/gpu/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dconv.log 2>&1 || { tail -40 $O/pytest_dconv.log; exit 1; }
tail -1 $O/pytest_dconv.log
timeout -k 10 180 python bench/conv_kernels.py --image 128 --batch 64 --reps 20 --json $O/per_launch.json > $O/per_launch.txt 2>&1 || { tail -30 $O/per_launch.txt; exit 1; }
MDT_CONV_DIRECT=0 timeout -k 10 180 python bench/conv_kernels.py --image 128 --batch 64 --reps 20 --json $O/per_launch_old.json > $O/per_launch_old.txt 2>&1 || { tail -30 $O/per_launch_old.txt; exit 1; }
paste <(grep -E "^ +[0-9]+ (igemm|thin|wgrad|launch_jobs|combine|reparam)" $O/per_launch_old.txt | cut -c1-45) <(grep -E "^ +[0-9]+ (igemm|thin|wgrad|launch_jobs|combine|reparam)" $O/per_launch.txt | cut -c1-45) | head -40
timeout -k 10 180 python3 bench.py --model conv128 --batch-size 64 --steps 50 --warmup 10 > $O/bench.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u -m pytest tests/gpu/test_conv_vae_kernels.py -q --timeout 120 --timeout-method thread > $O/pytest_cvk.log 2>&1 || { tail -40 $O/pytest_cvk.log; exit 1; }
tail -2 $O/pytest_cvk.log
