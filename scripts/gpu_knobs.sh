# A/B of the conv planner knobs (split-K depth, 64-row tile threshold, wgrad grid target)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs
mkdir -p $O
export TMPDIR=/tmp
run() {  # name model bs env...
  local name=$1 m=$2 bs=$3; shift 3
  env "$@" timeout -k 10 120 python3 bench.py --model $m --batch-size $bs --steps 300 --warmup 30 > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]); print('$name', d['ms_per_step'], d['config']['valid'])"
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run c28_new conv28 128 MDT_X=0 || exit 1
run c28_old conv28 128 MDT_CONV_SPLIT_KT_PER=4 MDT_CONV_SPLIT_MIN_KT=16 MDT_CONV_BM64_BELOW=512 MDT_CONV_WG_TARGET=320 || exit 1
run c28_new2 conv28 128 MDT_X=1 || exit 1
run c128_new conv128 64 MDT_X=0 || exit 1
run c128_old conv128 64 MDT_CONV_SPLIT_KT_PER=4 MDT_CONV_SPLIT_MIN_KT=16 MDT_CONV_BM64_BELOW=512 MDT_CONV_WG_TARGET=320 || exit 1
run c128_new2 conv128 64 MDT_X=1 || exit 1
run c128_w1024 conv128 64 MDT_CONV_WG_TARGET=1024 || exit 1
