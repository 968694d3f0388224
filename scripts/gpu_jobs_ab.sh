# fused job launches: correctness tests + A/B step time (+ timeline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/jobs
timeout -k 10 400 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_conv_igemm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/jobs/pytest.log 2>&1 || { tail -40 gpurun_out/jobs/pytest.log; exit 1; }
tail -3 gpurun_out/jobs/pytest.log
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  MDT_CONV_JOBS=0 timeout -k 10 120 python bench.py --model $m --batch-size $bs 2>/dev/null | grep metric > gpurun_out/jobs/${m}_unfused.json || exit 1
  MDT_CONV_JOBS=1 timeout -k 10 120 python bench.py --model $m --batch-size $bs 2>/dev/null | grep metric > gpurun_out/jobs/${m}_fused.json || exit 1
done
for f in gpurun_out/jobs/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
MODELS="conv28 conv128" bash scripts/gpu_timeline.sh > gpurun_out/jobs/timeline.log 2>&1 || exit 1
grep -E "kernels/step|median step" gpurun_out/jobs/timeline.log
