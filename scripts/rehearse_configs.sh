#!/bin/bash
# One-GPU rehearsal of the driver's 8-rank launches (BASELINE configs #3-#5):
# torch.distributed.run --nproc-per-node 8 bench.py --gpus 8 [--ngroups K]
# with all eight ranks sharing the box's one MI355X (gloo world: RCCL rejects
# two ranks per GPU; intra-group DDP forced to the fused xGMI jobs; every rank
# on its own 32-CU share). Correctness and plumbing only: eight processes
# time-share one GPU, so the throughput says nothing about an 8-GPU node.
#
# usage: scripts/rehearse_configs.sh OUTDIR   (run from the repo root)
set -o pipefail
out=${1:-gpurun_out/r5_configs}
mkdir -p "$out"
export DDP_BACKEND=gloo MDT_CU_SPLIT=1 MDT_REDUCER=xgmi MDT_P2P_TIMEOUT_S=${MDT_P2P_TIMEOUT_S:-20}
port=29711
for cfg in "cfg3 8 conv28 128" "cfg4 4 conv28 128" "cfg5 2 conv128 64"; do
  set -- $cfg
  tag=$1 K=$2 model=$3 bs=$4
  port=$((port + 1))
  echo "== $tag" >&2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 8 --ngroups "$K" --model "$model" --batch-size "$bs" --steps 20 \
    --warmup 5 --json-out "$out/$tag.json" > "$out/$tag.out" 2> "$out/$tag.err" || {
      rc=$?; echo "FAILED $tag rc=$rc" >&2; tail -30 "$out/$tag.err" >&2; exit $rc; }
  cat "$out/$tag.json"
done
