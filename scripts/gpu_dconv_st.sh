set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-dconv_st}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/gpu/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dconv.log 2>&1 || { tail -40 $O/pytest_dconv.log; exit 1; }
tail -1 $O/pytest_dconv.log
timeout -k 10 120 python bench/dconv_stamps.py --json $O/stamps.json > $O/stamps.txt 2>&1 || { tail -30 $O/stamps.txt; exit 1; }
grep -v amdgpu $O/stamps.txt
