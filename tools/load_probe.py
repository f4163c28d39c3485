"""Why is the trunk kernel slower inside the bench than isolated?  Times the cfg2 fp32 forward at
1,024 rows (pinned planes / outputs, 0.3 ms host gap between launches, ~70 % GPU duty like the
bench) for a sustained period, (a) with an idle host, then (b) with W processes doing random DRAM
gathers (like the engine threads' tree walks).  Prints the median kernel time per 5 s window.
GPU box only.  Usage: python tools/load_probe.py [--seconds 40] [--workers 14]
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hammer(stop, seed):
    rng = np.random.default_rng(seed)
    big = np.ones(1 << 27, dtype=np.float32)          # 512 MB per worker
    idx = rng.integers(0, big.size, size=1 << 22)
    s = 0.0
    while not stop.is_set():
        s += float(big[idx].sum())
    return s


def timed_window(net, seg, stream, seconds, torch):
    out = []
    t_end = time.time() + seconds
    win_t, win = time.time() + 5, []
    while time.time() < t_end:
        g = time.perf_counter() + 300e-6
        while time.perf_counter() < g:
            pass
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        net.forward_segments(stream.cuda_stream, seg)
        b.record(stream)
        b.synchronize()
        win.append(a.elapsed_time(b))
        if time.time() > win_t:
            out.append(float(np.median(win)))
            win, win_t = [], time.time() + 5
    return out


def main():
    import torch
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=40)
    ap.add_argument("--workers", type=int, default=14)
    args = ap.parse_args()
    desc = BASELINE_CONFIGS[2]["desc"]
    net = HipNet(desc, 0, "fp32")
    net.set_weights(to_blob(random_weights(desc, 3, bias_std=0.1)))
    stream = torch.cuda.Stream()
    n = 1024
    planes = torch.from_numpy(random_planes(desc, n, 9)).pin_memory()
    pols = [torch.empty((n, p), dtype=torch.float32).pin_memory() for p in desc.policy_dist_count]
    val = torch.empty((n, desc.num_values), dtype=torch.float32).pin_memory()
    seg = [(n, planes.data_ptr(), [p.data_ptr() for p in pols], val.data_ptr())]
    w = timed_window(net, seg, stream, args.seconds, torch)
    print("idle host:   " + " ".join("%.3f" % x for x in w), flush=True)
    ctx = mp.get_context("spawn")
    stop = ctx.Event()
    procs = [ctx.Process(target=hammer, args=(stop, i)) for i in range(args.workers)]
    for p in procs:
        p.start()
    time.sleep(3)
    w = timed_window(net, seg, stream, args.seconds, torch)
    stop.set()
    for p in procs:
        p.join(timeout=30)
    print("loaded host: " + " ".join("%.3f" % x for x in w), flush=True)
    net.close()


if __name__ == "__main__":
    main()
