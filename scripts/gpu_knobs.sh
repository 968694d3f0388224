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
run c28_t4 conv28 128 MDT_THIN_TCONV4=1 || exit 1
run c28_t1 conv28 128 MDT_X=0 || exit 1
run c28_t4b conv28 128 MDT_THIN_TCONV4=1 || exit 1
run c128_t4 conv128 64 MDT_THIN_TCONV4=1 || exit 1
run c128_t1 conv128 64 MDT_X=0 || exit 1
run c128_t4b conv128 64 MDT_THIN_TCONV4=1 || exit 1
