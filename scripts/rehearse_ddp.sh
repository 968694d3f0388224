#!/bin/bash
# One-GPU rehearsal of the shipped intra-group DDP path (BASELINE configs #4/#5):
# exactly the driver's N>1 bench launch (torch.distributed.run ... bench.py
# --gpus s --ngroups 1) with s ranks sharing the box's one MI355X. RCCL rejects
# two ranks on one GPU, so the world is gloo and the reducer is forced to the
# fused xGMI jobs (a gloo world otherwise resolves to c10d); MDT_CU_SPLIT=1 gives
# every rank a disjoint CU share so a rank spinning on a peer's flags can never
# hold the CUs that peer needs. Everything else stays at production defaults:
# graphs on, pair on, no split tail, no host barrier between push and reduce.
#
# usage: scripts/rehearse_ddp.sh OUTDIR [overlap...]   (run from the repo root)
set -o pipefail
out=${1:-gpurun_out/r5_rehearsal}
shift
overlaps=${*:-"0 1"}
mkdir -p "$out"
export MDT_CU_SPLIT=1 DDP_BACKEND=gloo MDT_REDUCER=xgmi MDT_P2P_TIMEOUT_S=${MDT_P2P_TIMEOUT_S:-10}
port=29611
for ov in $overlaps; do
  for cfg in "2 conv28 128" "4 conv28 128" "2 conv128 64" "4 conv128 64"; do
    set -- $cfg
    s=$1 model=$2 bs=$3
    tag="s${s}_${model}_ov${ov}"
    port=$((port + 1))
    echo "== $tag" >&2
    MDT_DDP_OVERLAP=$ov timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$s" \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$s" --ngroups 1 --model "$model" \
      --batch-size "$bs" --steps 20 --warmup 5 --json-out "$out/$tag.json" > "$out/$tag.out" 2> "$out/$tag.err" || {
        rc=$?; echo "FAILED $tag rc=$rc" >&2; tail -30 "$out/$tag.err" >&2; exit $rc; }
    cat "$out/$tag.json"
  done
done
