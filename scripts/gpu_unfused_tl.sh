# Diagnostic: kernel timeline of the conv28 step with every job as its own kernel (MDT_CONV_JOBS=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/unfused
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MDT_CONV_JOBS=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/ktimeline.py $f combine_reparam_k > $O/timeline_unfused_conv28.txt 2>&1 || true
cat $O/timeline_unfused_conv28.txt
