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
run c28_base conv28 128 MDT_X=0 || exit 1
run c28_kt1 conv28 128 MDT_CONV_SPLIT_KT_PER=1 || exit 1
run c28_kt2 conv28 128 MDT_CONV_SPLIT_KT_PER=2 || exit 1
run c28_minkt8_kt2 conv28 128 MDT_CONV_SPLIT_MIN_KT=8 MDT_CONV_SPLIT_KT_PER=2 || exit 1
run c28_minkt8_kt1 conv28 128 MDT_CONV_SPLIT_MIN_KT=8 MDT_CONV_SPLIT_KT_PER=1 || exit 1
run c28_wg640 conv28 128 MDT_CONV_WG_TARGET=640 || exit 1
run c28_wg160 conv28 128 MDT_CONV_WG_TARGET=160 || exit 1
run c28_bm1024 conv28 128 MDT_CONV_BM64_BELOW=1024 || exit 1
run c28_base2 conv28 128 MDT_X=1 || exit 1
run c128_base conv128 64 MDT_X=0 || exit 1
run c128_bm1024 conv128 64 MDT_CONV_BM64_BELOW=1024 || exit 1
run c128_bm2048 conv128 64 MDT_CONV_BM64_BELOW=2048 || exit 1
run c128_wg640 conv128 64 MDT_CONV_WG_TARGET=640 || exit 1
run c128_wg1024 conv128 64 MDT_CONV_WG_TARGET=1024 || exit 1
run c128_kt2 conv128 64 MDT_CONV_SPLIT_KT_PER=2 || exit 1
run c128_base2 conv128 64 MDT_X=1 || exit 1
