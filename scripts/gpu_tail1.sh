# One-launch optimizer tail: bitwise tests, then bench A/B (MDT_CONV_TAIL1=1 default vs 0), kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tail2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/gpu/test_conv_vae_kernels.py tests/gpu/test_grad_finalize.py -x -v --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1 || { tail -40 $O/pytest_conv.log; exit 1; }
tail -3 $O/pytest_conv.log
run() {  # name model bs env...
  local name=$1 m=$2 bs=$3; shift 3
  env "$@" timeout -k 10 120 python3 bench.py --model $m --batch-size $bs --steps 300 --warmup 30 > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]); print('$name', d['ms_per_step'], d['config']['valid'])"
}
run c28_sp conv28 128 MDT_CONV_SPREAD_FIN=1 || exit 1
run c28_nosp conv28 128 MDT_CONV_SPREAD_FIN=0 || exit 1
run c28_sp_t1 conv28 128 MDT_CONV_TAIL1=1 || exit 1
run c28_sp2 conv28 128 MDT_CONV_SPREAD_FIN=1 || exit 1
run c28_nosp2 conv28 128 MDT_CONV_SPREAD_FIN=0 || exit 1
run c128_sp conv128 64 MDT_CONV_SPREAD_FIN=1 || exit 1
run c128_nosp conv128 64 MDT_CONV_SPREAD_FIN=0 || exit 1
run c128_sp2 conv128 64 MDT_CONV_SPREAD_FIN=1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 40 --warmup 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); echo trace $f
python3 scripts/ktimeline.py $f combine_reparam_k > $O/timeline.txt 2>&1 || true
tail -20 $O/timeline.txt
