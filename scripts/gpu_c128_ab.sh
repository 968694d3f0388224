# conv128 step A/B: direct kernels on/off, two-stream backward on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-c128ab}
mkdir -p $O
for cfg in "1 0" "1 1" "0 0" "0 1"; do
set -- $cfg
for b in 64 128; do
MDT_CONV_DIRECT=$1 MDT_CONV_OVERLAP=$2 timeout -k 10 180 python3 bench.py --model conv128 --batch-size $b --steps 50 --warmup 10 > $O/b_$1_$2_$b.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
python -c "import json;d=json.load(open('$O/b_$1_$2_$b.json'));print('direct=$1 overlap=$2 B=$b', d['ms_per_step'], 'ms', d['value'])"
done
done
MDT_CONV_OVERLAP=1 timeout -k 10 180 python bench/conv_kernels.py --image 128 --batch 64 --reps 20 --json $O/per_launch.json > $O/per_launch.txt 2>&1 || { tail -30 $O/per_launch.txt; exit 1; }
grep -E "^ +[0-9]+ " $O/per_launch.txt | grep -v " 1\.[0-9][0-9] us\| 0\.[0-9][0-9] us" | cut -c1-60
