# A/B: column-tile split for shallow GEMMs with tiny grids (decoder Linear fwd, encoder head dgrad)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bnshallow
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for cfg in "16 512" "1 64" "1 128" "1 256"; do
    set -- $cfg
    MDT_CONV_BN_SPLIT_MIN_KT=$1 MDT_CONV_BN_SPLIT_BELOW=$2 MDT_JOBS_DEBUG=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28.json 2>$O/err_$1_$2.txt || { tail -20 $O/err_$1_$2.txt; exit 1; }
    echo "conv28 rep$rep min_kt=$1 below=$2 $(python -c "import json;d=json.load(open('$O/c28.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
grep -h "\[jobs\]" $O/err_*.txt | sort | uniq -c || true
