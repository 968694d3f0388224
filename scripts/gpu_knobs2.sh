# Planner knob re-sweep (conv28) on top of the current defaults (deferred transposes,
# spread finalize, tiny-grid column split)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs2
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for kv in "BASE=1" "MDT_CONV_WG_TARGET=96" "MDT_CONV_WG_TARGET=128" "MDT_CONV_WG_TARGET=240" "MDT_CONV_BM64_BELOW=512" "MDT_CONV_BM64_BELOW=2048" "MDT_CONV_SPLIT_MIN_KT=4" "MDT_CONV_SPLIT_MIN_KT=16" "MDT_CONV_BN_SPLIT_TINY=40" "MDT_CONV_BN_SPLIT_TINY=100" "MDT_CONV_SPLIT_KT_PER=2"; do
    env $kv timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv28 rep$rep $kv $(python -c "import json;d=json.load(open('$O/c28.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
