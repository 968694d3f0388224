"""
Concurrent VAE hyper-parameter search over K process groups (MI355X-native).

Drop-in for /root/reference/vae-hpo.py: same flags and defaults
(``--batch-size 128 --epochs 3 --ngroups 2``), same stdout lines, same
``results-{group_rank}/`` images, same schedule (trial g trains epochs+g
epochs). Launch one process per GPU with any launcher the reference supports
(jsrun / srun / mpirun) or torchrun / ``python -m multidisttorch_amd.launch``.

Extensions (opt-in, default output unchanged): ``--lr`` / ``--beta`` (scalar or
comma list, one per trial), ``--seed``, ``--ckpt-dir`` + ``--resume``,
``--metrics-dir`` (JSONL + aggregate samples/s), ``--per-group-results``, ``--bucket-mb``,
``--no-graphs``, ``--backend {hip,torch}``, ``--synthetic/--real-data``,
``--trials-per-group T`` (T concurrent trials per single-rank group, one HIP
stream each: trial packing on MI355X).
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from utils import *  # noqa: F401,F403  (reference-compatible API + re-exports)

from multidisttorch_amd.hpo.runner import RunOptions, idle_rank, run_packed_trials, run_trial
from multidisttorch_amd.hpo.trial import build_specs, parse_list
from multidisttorch_amd.parallel.autotune import parse_bucket_mb
from multidisttorch_amd.runtime.bootstrap import control_group
from multidisttorch_amd.runtime.faults import create_health_groups


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="VAE MNIST Example")
    parser.add_argument("--batch-size", type=int, default=128, metavar="N",
                        help="input batch size for training (default: 128)")
    parser.add_argument("--epochs", type=int, default=3, metavar="N",
                        help="number of epochs to train (default: 1)")
    parser.add_argument("--ngroups", type=int, help="number of groups", default=2)
    # ---- extensions ----
    parser.add_argument("--lr", type=str, default=None, help="learning rate(s), comma list per trial")
    parser.add_argument("--beta", type=str, default=None, help="KLD weight(s), comma list per trial")
    parser.add_argument("--seed", type=int, default=0, help="base seed (trial g uses seed+g)")
    parser.add_argument("--no-epoch-offset", action="store_true", help="all trials train --epochs epochs")
    parser.add_argument("--log-interval", type=int, default=10)
    parser.add_argument("--ckpt-dir", type=str, default=None)
    parser.add_argument("--resume", action="store_true")
    parser.add_argument("--metrics-dir", type=str, default=None)
    parser.add_argument("--per-group-results", action="store_true")
    parser.add_argument("--no-results", action="store_true", help="skip PNG writing")
    parser.add_argument("--no-graphs", action="store_true")
    parser.add_argument("--graph-steps", type=int, default=10)
    parser.add_argument("--backend", type=str, default=None, choices=[None, "hip", "torch"])
    parser.add_argument("--real-data", action="store_true", help="require MNIST IDX files under --data-dir")
    parser.add_argument("--synthetic", action="store_true",
                        help="always use the synthetic MNIST-shaped set (default: IDX files under --data-dir "
                             "or data-dir/MNIST/raw when present, synthetic otherwise)")
    parser.add_argument("--data-dir", type=str, default="data")
    parser.add_argument("--train-samples", type=int, default=None)
    parser.add_argument("--test-samples", type=int, default=None)
    parser.add_argument("--model", type=str, default="mlp", choices=["mlp", "conv"],
                        help="mlp = reference MLP-VAE (fp32); conv = bf16 conv/deconv VAE")
    parser.add_argument("--image-size", type=int, default=28, choices=[28, 128])
    parser.add_argument("--dtype", type=str, default=None, choices=[None, "fp32", "bf16"],
                        help="compute dtype; mlp runs fp32 (the reference's precision), conv runs bf16 MFMA")
    parser.add_argument("--profile", action="store_true",
                        help="roctx ranges around phases (rocprofv3 --marker-trace) + synced phase timings in metrics")
    parser.add_argument("--debug-sync", action="store_true",
                        help="serialize every kernel launch (AMD_SERIALIZE_KERNEL=3): race / fault triage")
    parser.add_argument("--trials-per-group", type=int, default=1,
                        help="train T trials concurrently per (single-rank) group, one HIP stream each")
    parser.add_argument("--bucket-mb", type=str, default=None,
                        help="intra-group all-reduce buckets: MiB cap, 0 = one bucket, 'auto' = measured")
    return parser.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    from multidisttorch_amd.runtime.env import apply_cu_split

    apply_cu_split()  # one-GPU multi-rank rehearsals only (MDT_CU_SPLIT=1), before HIP initialises
    if args.debug_sync:  # must precede any HIP initialisation
        os.environ["AMD_SERIALIZE_KERNEL"] = "3"
        os.environ["AMD_SERIALIZE_COPY"] = "3"
    want = {"mlp": "fp32", "conv": "bf16"}[args.model]
    if args.dtype is not None and args.dtype != want:
        raise SystemExit(f"--model {args.model} computes in {want} (requested {args.dtype})")
    if args.profile:
        from multidisttorch_amd.obs import trace

        trace.enable()
        if args.metrics_dir is None:
            args.metrics_dir = "metrics"
    ngroups = args.ngroups
    comm_size, rank = setup_ddp()
    processes_groups = setup_ddp_groups(ngroups)
    control_group()  # world collective: create the gloo control plane on every rank
    create_health_groups(ngroups)  # world collective: per-trial gloo health agreement (faults.py)

    T = max(1, args.trials_per_group)
    specs = build_specs(ngroups * T, args.epochs, parse_list(args.lr), parse_list(args.beta), args.seed,
                        epoch_offset=not args.no_epoch_offset)
    opts = RunOptions(batch_size=args.batch_size, log_interval=args.log_interval,
                      backend=args.backend, use_graphs=not args.no_graphs, graph_steps=args.graph_steps,
                      ckpt_dir=args.ckpt_dir, resume=args.resume, metrics_dir=args.metrics_dir,
                      results=not args.no_results, per_group_results=args.per_group_results,
                      train_samples=args.train_samples, test_samples=args.test_samples,
                      data_dir=args.data_dir,
                      synthetic=False if args.real_data else (True if args.synthetic else None),
                      model=args.model, image_size=args.image_size, bucket_mb=parse_bucket_mb(args.bucket_mb),
                      profile=args.profile)
    results = []
    member = False
    for group_id, group in enumerate(processes_groups):
        if dist.get_rank(group) >= 0:
            member = True
            if T == 1:
                results.append(run_trial(specs[group_id], group, opts))
            else:
                results.extend(run_packed_trials(specs[group_id * T:(group_id + 1) * T], group, opts,
                                                 num_trials=ngroups * T))
    if not member:
        idle_rank()

    # aggregate samples/s: samples once per trial, max wall over ranks
    mine = [(r.group_id, r.samples, r.wall_s, r.failed) for r in results]
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, mine, group=control_group())
    if dist.get_rank() == 0:
        per_trial, wall, failed = {}, 0.0, set()
        for lst in gathered:
            for gid, samples, w, bad in lst or []:
                per_trial[gid] = min(per_trial.get(gid, samples), samples)
                wall = max(wall, w)
                if bad:
                    failed.add(gid)
        summary = {"metric": "aggregate VAE samples/sec across K concurrent HPO trials",
                   "trials": len(per_trial), "samples": int(sum(per_trial.values())),
                   "wall_s": round(wall, 4),
                   "value": round(sum(per_trial.values()) / max(wall, 1e-9), 1), "unit": "samples/s",
                   "failed_trials": sorted(failed)}
        if args.metrics_dir:
            os.makedirs(args.metrics_dir, exist_ok=True)
            with open(os.path.join(args.metrics_dir, "aggregate.json"), "w") as f:
                json.dump(summary, f)
        print("MDT_AGGREGATE " + json.dumps(summary), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
