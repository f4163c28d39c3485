"""Split the fused forward's time into trunk and fixed (input + initial conv + heads) parts by timing
the cfg2 geometry at several residual-block counts: slope = time per residual block (2 convs),
intercept = everything else.  GPU box only.

Usage: python tools/kernel_breakdown.py [--variants 12,13] [--batches 256,1024] [--precision fp32] [--pinned]
--pinned: planes and outputs in pinned host memory (the runner's zero-copy path), timed with events
around a segmented launch, instead of gz_net_forward's device staging.
"""
import argparse
import dataclasses
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402


def staged_times(net, x, reps):
    net.forward(x)
    ts = []
    for _ in range(reps):
        net.forward(x)
        ts.append(net.last_kernel_ms())
    return ts


def pinned_times(net, desc, x, reps):
    import torch
    n = x.shape[0]
    planes = torch.from_numpy(x).pin_memory()
    pols = [torch.empty((n, p), dtype=torch.float32).pin_memory() for p in desc.policy_dist_count]
    val = torch.empty((n, desc.num_values), dtype=torch.float32).pin_memory()
    stream = torch.cuda.Stream()
    seg = [(n, planes.data_ptr(), [p.data_ptr() for p in pols], val.data_ptr())]
    ts = []
    for i in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        net.forward_segments(stream.cuda_stream, seg)
        b.record(stream)
        b.synchronize()
        if i:
            ts.append(a.elapsed_time(b))
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--variants", default="12")
    ap.add_argument("--batches", default="256,1024")
    ap.add_argument("--blocks", default="0,1,2,6")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--pinned", action="store_true")
    args = ap.parse_args()
    base = BASELINE_CONFIGS[args.cfg]["desc"]
    for v in args.variants.split(","):
        os.environ["GZ_KERNEL_VARIANT"] = v
        for n in [int(b) for b in args.batches.split(",")]:
            xs, ys = [], []
            for nb in [int(b) for b in args.blocks.split(",")]:
                desc = dataclasses.replace(base, residual_layers=nb)
                net = HipNet(desc, 0, args.precision)
                net.set_weights(to_blob(random_weights(desc, 3, bias_std=0.1)))
                x = random_planes(desc, n, 9)
                ts = pinned_times(net, desc, x, args.reps) if args.pinned else staged_times(net, x, args.reps)
                net.close()
                xs.append(nb)
                ys.append(float(np.median(ts)) * 1e3)
                print("variant %s N=%d blocks=%d  %.1f us" % (v, n, nb, ys[-1]), flush=True)
            os.environ["GZ_KERNEL_STAMPS"] = "1"
            desc = base
            net = HipNet(desc, 0, args.precision)
            net.set_weights(to_blob(random_weights(desc, 3, bias_std=0.1)))
            net.forward(random_planes(desc, n, 9))
            st = net.stamp_avg()
            net.close()
            del os.environ["GZ_KERNEL_STAMPS"]
            print("variant %s N=%d trunk-kernel stamps (cycles per workgroup): input+conv0 %.0f, residual trunk %.0f, "
                  "head 1x1 convs + features %.0f, dense heads %.0f" % ((v, n) + tuple(st[1:5])), flush=True)
            slope, icpt = np.polyfit(xs, ys, 1)
            conv_flops = 2 * base.hw * base.cnn_filter_size ** 2 * 9 * 2 * n
            print("variant %s N=%d: %.1f us per residual block (%.0f TFLOP/s in the trunk), %.1f us fixed"
                  % (v, n, slope, conv_flops / slope / 1e6, icpt), flush=True)


if __name__ == "__main__":
    main()
