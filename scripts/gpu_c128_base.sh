# conv128 B=64: per-launch times, driver-style bench, kernel trace of the graph step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-c128}
mkdir -p $O
timeout -k 10 180 python bench/conv_kernels.py --image 128 --batch 64 --reps 20 --json $O/per_launch.json > $O/per_launch.txt 2>&1 || { tail -30 $O/per_launch.txt; exit 1; }
grep -v amdgpu.ids $O/per_launch.txt | tail -45
timeout -k 10 180 python3 bench.py --model conv128 --batch-size 64 --steps 50 --warmup 10 > $O/bench.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o c128 -- python3 $GRAFT_REPO_ROOT/bench.py --model conv128 --batch-size 64 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
