set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-dconv_ab}
mkdir -p $O
for alt in 0 1; do
MDT_DCONV_ALT=$alt timeout -k 10 200 python -u -m pytest tests/gpu/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dconv_$alt.log 2>&1 || { tail -40 $O/pytest_dconv_$alt.log; exit 1; }
tail -1 $O/pytest_dconv_$alt.log
MDT_DCONV_ALT=$alt timeout -k 10 120 python bench/dconv_stamps.py --json $O/stamps_$alt.json > $O/stamps_$alt.txt 2>&1 || { tail -30 $O/stamps_$alt.txt; exit 1; }
grep -v amdgpu $O/stamps_$alt.txt
MDT_DCONV_ALT=$alt timeout -k 10 120 python bench/dconv_stamps.py --batch 128 > $O/stamps128_$alt.txt 2>&1 || { tail -30 $O/stamps128_$alt.txt; exit 1; }
grep -v amdgpu $O/stamps128_$alt.txt | cut -c1-90
done
