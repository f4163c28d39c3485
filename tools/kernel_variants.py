"""Time every compiled forward-kernel variant (GZ_KERNEL_VARIANT) on the BASELINE geometries.

Usage (GPU box): python tools/kernel_variants.py [--batches 256,1024] [--reps 20]
Prints one line per (config, variant, batch): median event-timed kernel ms, TFLOP/s, and the max
abs difference of every output against the default variant (results must be batch-invariant and
identical up to fp32 summation order).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402

VARIANTS = ["default", "12", "11", "21"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="256,1024")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default="1,2,3")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--precision", default="bf16", choices=["bf16", "bf16x3", "split", "fp32"])
    args = ap.parse_args()
    batches = [int(b) for b in args.batches.split(",")]
    for cfg in [int(c) for c in args.configs.split(",")]:
        desc = BASELINE_CONFIGS[cfg]["desc"]
        w = to_blob(random_weights(desc, 11, bias_std=0.1))
        xs = {n: random_planes(desc, n, 5 + n) for n in batches}
        base = {}
        for v in args.variants.split(","):
            if v == "default":        # the library's per-launch dispatch
                os.environ.pop("GZ_KERNEL_VARIANT", None)
            else:
                os.environ["GZ_KERNEL_VARIANT"] = v
            try:
                net = HipNet(desc, 0, args.precision)
            except RuntimeError as e:
                print("cfg%d variant %s: n/a (%s)" % (cfg, v, e), flush=True)
                continue
            net.set_weights(w)
            fl = net.flops_per_eval()
            for n in batches:
                out = net.forward(xs[n])
                ts = []
                for _ in range(args.reps):
                    net.forward(xs[n])
                    ts.append(net.last_kernel_ms())
                ms = float(np.median(ts))
                if n not in base:
                    base[n] = out
                diff = max(float(np.abs(a - b).max()) for a, b in zip(out, base[n]))
                print("cfg%d %s variant %s N=%5d  %8.3f ms  %7.1f TFLOP/s  %9.0f evals/s  maxdiff %.2e"
                      % (cfg, args.precision, v, n, ms, fl * n / ms / 1e9, n / ms * 1e3, diff), flush=True)
            net.close()


if __name__ == "__main__":
    main()
