set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m multidisttorch_amd.obs.probe --json gpurun_out/probe.json > gpurun_out/probe.log 2>&1; rc=$?
cat gpurun_out/probe.log | tail -20
exit $rc
