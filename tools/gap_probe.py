"""Does an idle gap between launches slow the next trunk kernel?  Times the cfg2 forward (pinned
planes, as the runner's launches) back to back and with a host-side gap before each launch, for
several launch sizes.  GPU box only.

Usage: python tools/gap_probe.py [--precision fp32] [--rows 512,1024,1536] [--gaps-us 0,300,1000]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"])
    ap.add_argument("--rows", default="512,1024,1536")
    ap.add_argument("--gaps-us", default="0,300,1000,3000")
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--weight-seed", type=int, default=3)
    ap.add_argument("--bias-std", type=float, default=0.1)
    args = ap.parse_args()
    desc = BASELINE_CONFIGS[2]["desc"]
    net = HipNet(desc, 0, args.precision)
    net.set_weights(to_blob(random_weights(desc, args.weight_seed, bias_std=args.bias_std)))
    stream = torch.cuda.Stream()
    for n in [int(r) for r in args.rows.split(",")]:
        planes = torch.from_numpy(random_planes(desc, n, 9)).pin_memory()
        pols = [torch.empty((n, p), dtype=torch.float32).pin_memory() for p in desc.policy_dist_count]
        val = torch.empty((n, desc.num_values), dtype=torch.float32).pin_memory()
        seg = [(n, planes.data_ptr(), [p.data_ptr() for p in pols], val.data_ptr())]
        for gap in [int(g) for g in args.gaps_us.split(",")]:
            ts = []
            for i in range(args.reps + 2):
                if gap:
                    t_end = time.perf_counter() + gap * 1e-6
                    while time.perf_counter() < t_end:
                        pass
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                net.forward_segments(stream.cuda_stream, seg)
                b.record(stream)
                if gap:
                    b.synchronize()
                    if i >= 2:
                        ts.append(a.elapsed_time(b))
                else:
                    ts.append((a, b))
            if not gap:
                torch.cuda.synchronize()
                ts = [a.elapsed_time(b) for a, b in ts[2:]]
            print("w%d/b%.2f %s rows %5d gap %5d us: median %.3f ms  min %.3f  max %.3f"
                  % (args.weight_seed, args.bias_std, args.precision, n, gap, np.median(ts), np.min(ts), np.max(ts)), flush=True)
    net.close()


if __name__ == "__main__":
    main()
