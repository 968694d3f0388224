# two-stream conv backward: correctness tests + A/B step time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ovl
timeout -k 10 300 python -u -m pytest tests/gpu/test_conv_vae_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ovl/pytest.log 2>&1 || { tail -40 gpurun_out/ovl/pytest.log; exit 1; }
tail -3 gpurun_out/ovl/pytest.log
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  MDT_CONV_OVERLAP=0 timeout -k 10 120 python bench.py --model $m --batch-size $bs > gpurun_out/ovl/${m}_seq.json 2>/dev/null || exit 1
  MDT_CONV_OVERLAP=1 timeout -k 10 120 python bench.py --model $m --batch-size $bs > gpurun_out/ovl/${m}_ovl.json 2>/dev/null || exit 1
done
for f in gpurun_out/ovl/*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'])"; done
