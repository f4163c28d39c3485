"""Kernel time of one forward launch of a BASELINE config's net at n rows, per precision
(net.last_kernel_ms: HIP events around the launch)."""
import argparse
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--rows", type=int, default=1024)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--precision", default="bf16,fp32")
a = ap.parse_args()
desc = BASELINE_CONFIGS[a.config]["desc"]
w = to_blob(random_weights(desc, 7921))
x = random_planes(desc, a.rows, 1)
for prec in a.precision.split(","):
    net = HipNet(desc, 0, prec)
    net.set_weights(w)
    ms = []
    for _ in range(a.reps):
        net.forward(x)
        ms.append(net.last_kernel_ms())
    best = min(ms[1:]) if len(ms) > 1 else ms[0]
    tf = desc.flops_per_eval() * a.rows / (best * 1e-3) / 1e12
    mult = 3 if prec == "fp32" else 1
    print("cfg%d %s rows %d: kernel %.3f ms (all %s) -> %.1f TFLOP/s algorithmic, %.1f issued (x%d)"
          % (a.config, prec, a.rows, best, ["%.3f" % m for m in ms], tf, tf * mult, mult), flush=True)
