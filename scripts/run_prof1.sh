set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/prof1/bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
find gpurun_out/prof1 -name "*stats*" | head; 
exit $rc
