# p2p (hipIpc one-shot) reducer tests + the RCCL reducer tests (shared StreamBuckets base)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/p2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/gpu/test_p2p_reducer.py tests/gpu/test_rccl_reducer.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -40 $O/pytest.log
exit $rc
