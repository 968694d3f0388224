# Rehearse the driver's N>1 bench launch on the 1-GPU box (both ranks share cuda:0, so this
# checks the launch / barrier / max-over-ranks / JSON contract, not scaling), then a csv
# kernel-stats profile of the headline step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/n2
mkdir -p $O
DDP_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29931 bench.py --gpus 2 --steps 100 --warmup 10 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -30 $O/bench_n2_gloo.err; exit 1; }
cat $O/bench_n2_gloo.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29932 bench.py --gpus 2 --steps 100 --warmup 10 > $O/bench_n2_nccl.json 2> $O/bench_n2_nccl.err || { tail -30 $O/bench_n2_nccl.err; exit 1; }
cat $O/bench_n2_nccl.json
