# MDT_CONV_DEFER_WT: bitwise GPU tests, then bench A/B (interleaved repeats) and a kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/defer
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/gpu/test_conv_vae_kernels.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/ab.txt
for rep in 1 2 3; do
  for d in 0 1 2; do
    MDT_CONV_DEFER_WT=$d MDT_JOBS_DEBUG=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28_d$d.json 2>$O/err_c28_d$d.txt || { tail -20 $O/err_c28_d$d.txt; exit 1; }
    echo "conv28 rep$rep defer=$d $(python -c "import json;d=json.load(open('$O/c28_d$d.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
for rep in 1 2; do
  for d in 0 1 2; do
    MDT_CONV_DEFER_WT=$d MDT_JOBS_DEBUG=1 timeout -k 10 120 python bench.py --model conv128 --batch-size 64 --steps 300 --warmup 30 > $O/c128_d$d.json 2>$O/err_c128_d$d.txt || { tail -20 $O/err_c128_d$d.txt; exit 1; }
    echo "conv128 B=64 rep$rep defer=$d $(python -c "import json;d=json.load(open('$O/c128_d$d.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done


cd /tmp && export TMPDIR=/tmp
MDT_CONV_DEFER_WT=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/ktimeline.py $f combine_reparam_k > $O/timeline_defer_conv28.txt 2>&1 || true
head -25 $O/timeline_defer_conv28.txt
grep -h "\[jobs\]" $O/err_*.txt | sort | uniq -c || true
