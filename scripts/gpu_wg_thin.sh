# A/B of MDT_CONV_WG_TARGET_THIN (m-split grid of the single-channel wgrad layers),
# plus the N=2 torchrun bench rehearsal after the timing-barrier change and an 8-trial
# packed run (every default-sweep (lr, beta) point stays finite over 330 steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wgthin
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for t in 0 8 16 32 64; do
    MDT_CONV_WG_TARGET_THIN=$t timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/c28_t$t.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "conv28 rep$rep thin_target=$t $(python -c "import json;d=json.load(open('$O/c28_t$t.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
  done
done
for t in 0 16 32 64; do
  MDT_CONV_WG_TARGET_THIN=$t timeout -k 10 120 python bench.py --model conv128 --batch-size 64 --steps 300 --warmup 30 > $O/c128_t$t.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
  echo "conv128 B=64 thin_target=$t $(python -c "import json;d=json.load(open('$O/c128_t$t.json'));print(d['ms_per_step'], d['config']['valid'])")" | tee -a $O/ab.txt
done
timeout -k 10 180 python bench.py --trials-per-gpu 8 --steps 300 --warmup 30 > $O/pack8.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/pack8.json
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29941 bench.py --gpus 2 --steps 100 --warmup 10 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
