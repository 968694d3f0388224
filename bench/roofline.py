#!/usr/bin/env python3
"""Compulsory-traffic / MFMA roofline of one conv-VAE training step on MI355X.

For every layer op of the step (forward, backward-data, weight gradient) and
the optimizer tail, count the FLOPs and the bytes that MUST cross HBM (each
operand read once, each result written once: bf16 NHWC activations and
activation gradients, bf16 weights, f32 weight gradients, Adam's f32 p/m/v),
and price them at the chip's dense bf16 MFMA peak and at a sustained HBM
rate. The floor of an op is max(MFMA time, HBM time); a kernel far above its
floor is latency/occupancy-bound, one near it can only get faster by moving
fewer bytes. Optionally joins a rocprofv3 kernel-trace summary (per-step
kernel times, from ``scripts/kstats.py``) for the measured column.

    python bench/roofline.py [--image 128] [--batch 64] [--hbm-tbs 5.0] [--mfma-pfs 2.5]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def layer_ops(spec, B):
    """(name, flops, bytes) per op; activations bf16, weight gradients f32."""
    ops = []
    for i, l in enumerate(spec):
        if l.kind == "linear":
            xin, xout = l.cin, l.cout
            macs = B * l.cin * l.cout
            wbytes = 2 * l.cin * l.cout
        else:
            xin = l.in_hw * l.in_hw * l.cin
            xout = l.out_hw * l.out_hw * l.cout
            if l.kind == "conv":
                macs = B * l.out_hw * l.out_hw * l.cout * l.k * l.k * l.cin
            else:  # transposed conv: each input pixel scatters k*k taps
                macs = B * l.in_hw * l.in_hw * l.cin * l.k * l.k * l.cout
            wbytes = 2 * l.k * l.k * l.cin * l.cout
        a_in, a_out = 2 * B * xin, 2 * B * xout
        wn = wbytes // 2
        ops.append((f"{l.name} fwd", 2 * macs, a_in + a_out + wbytes))
        if i > 0:  # backward-data: read dY (+ the input activation as ReLU mask), write dX
            ops.append((f"{l.name} dgrad", 2 * macs, a_out + 2 * a_in + wbytes))
        ops.append((f"{l.name} wgrad", 2 * macs, a_out + a_in + 4 * wn))
    return ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", type=int, default=128)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hbm-tbs", type=float, default=5.0, help="sustained HBM rate used for the floor (TB/s)")
    ap.add_argument("--mfma-pfs", type=float, default=2.5, help="dense bf16 MFMA peak (PFLOP/s)")
    ap.add_argument("--measured-us", type=float, default=None, help="measured step time to compare against")
    a = ap.parse_args()
    import torch
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, _w_shape

    tr = ConvVaeTrainer(batch_size=a.batch, image=a.image, z=32 if a.image == 28 else 64,
                        device=torch.device("cpu"), backend="torch")
    ops = layer_ops(tr.spec, a.batch)
    nparam = sum(math.prod(_w_shape(l)) + l.cout for l in tr.spec)
    # Adam: read g, p, m, v; write p, m, v (f32) + the bf16 weight copy
    ops.append(("optimizer (Adam + bf16 cast)", 0, nparam * (4 * 4 + 3 * 4 + 2)))
    hbm, mf = a.hbm_tbs * 1e12, a.mfma_pfs * 1e15
    tot_f = tot_b = tot_floor = 0.0
    print(f"{'op':32s} {'GFLOP':>7s} {'MB':>7s} {'MFMA us':>8s} {'HBM us':>7s} {'floor':>6s}  bound")
    for name, f, b in ops:
        tm, tb = f / mf * 1e6, b / hbm * 1e6
        fl = max(tm, tb)
        tot_f += f
        tot_b += b
        tot_floor += fl
        print(f"{name:32s} {f / 1e9:7.2f} {b / 1e6:7.1f} {tm:8.2f} {tb:7.2f} {fl:6.2f}  {'MFMA' if tm > tb else 'HBM'}")
    print(f"{'step total':32s} {tot_f / 1e9:7.2f} {tot_b / 1e6:7.1f} {tot_f / mf * 1e6:8.2f} {tot_b / hbm * 1e6:7.2f} "
          f"{tot_floor:6.2f}")
    print(f"params {nparam}; arithmetic intensity {tot_f / tot_b:.0f} FLOP/B (ridge at these rates: {mf / hbm:.0f})")
    print(f"MFMA-busy ceiling if every op ran at its floor: {100 * tot_f / mf * 1e6 / tot_floor:.0f} %")
    if a.measured_us:
        print(f"measured {a.measured_us:.1f} us = {a.measured_us / tot_floor:.2f} x the floor; MFMA busy "
              f"{100 * tot_f / mf * 1e6 / a.measured_us:.1f} %")


if __name__ == "__main__":
    main()
