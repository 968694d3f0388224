set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m multidisttorch_amd.obs.stamps --json gpurun_out/stamps.json > gpurun_out/stamps.log 2>&1; rc=$?
python multidisttorch_amd/obs/show_stamps.py
exit $rc
