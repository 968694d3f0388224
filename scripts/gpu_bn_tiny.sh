# MDT_CONV_BN_SPLIT_TINY default (64) vs off (0): conv GPU tests, interleaved bench A/B, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bn_tiny
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_conv_igemm.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/ab.txt
for rep in 1 2 3; do
  for t in 0 64; do
    MDT_CONV_BN_SPLIT_TINY=$t MDT_JOBS_DEBUG=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28_t$t.json 2>$O/err_c28_$t.txt || { tail -20 $O/err_c28_$t.txt; exit 1; }
    echo "conv28 rep$rep tiny=$t $(python -c "import json;d=json.load(open('$O/c28_t$t.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
for rep in 1 2; do
  for t in 0 64; do
    MDT_CONV_BN_SPLIT_TINY=$t MDT_JOBS_DEBUG=1 timeout -k 10 120 python bench.py --model conv128 --batch-size 64 --steps 300 --warmup 30 > $O/c128_t$t.json 2>$O/err_c128_$t.txt || { tail -20 $O/err_c128_$t.txt; exit 1; }
    echo "conv128 B=64 rep$rep tiny=$t $(python -c "import json;d=json.load(open('$O/c128_t$t.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
grep -h "\[jobs\]" $O/err_*.txt | sort | uniq -c || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/ktimeline.py $f combine_reparam_k > $O/timeline_conv28.txt 2>&1 || true
head -20 $O/timeline_conv28.txt
