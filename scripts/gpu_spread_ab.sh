# A/B: spread finalize on top of the deferred transposes (conv28 and conv128 B=64)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/spread2
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for s in 0 1; do
    MDT_CONV_SPREAD_FIN=$s timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28_s$s.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv28 rep$rep spread=$s $(python -c "import json;d=json.load(open('$O/c28_s$s.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
