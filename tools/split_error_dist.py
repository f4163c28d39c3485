"""Error distribution of the bf16x3 split forward (the bench's arithmetic) against the float64
oracle, on bench.py's own weights (random_weights(desc, 7921), undamped), at the bench's launch
shape: >= 1,024-row launches of several pinned-host segments (exactly as the runner issues them),
for cfg2 and for each deep config in its bench mode; one launch per input seed.

The oracle is oracle/nn_ref_torch.py (nn_ref.forward restated in float64 torch, run on the GPU;
pinned to nn_ref by tests/test_nn_oracle.py).  Writes one JSON document: per config and seed the
max / mean |error| of the probabilities (policies + value), the max per-row KL(oracle || kernel) and
the heads' logits error relative to max(1, max |oracle logit|).  galvanise_zero_amd/nn/tolerance.py
states each config's tolerance from the committed result (>= 3x the maximum over the seeds).

usage: python tools/split_error_dist.py OUT.json [--seeds 10] [--configs cfg2,cfg3,cfg4,cfg5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

# config: (BASELINE index, precision, rows per launch, segment sizes pattern)
CONFIGS = {
    "cfg2": (2, "fp32", 1103),
    "cfg3": (3, "fp32", 1103),
    "cfg4": (4, "fp32", 1024),
    "cfg5": (5, "fp32", 1024),
}


def segments(n, rng):
    """Pool-sized segments (~200-256 rows, the first starting mid-pool like a split batch's
    remainder) adding up to n."""
    out = []
    left = n
    while left > 0:
        k = int(min(left, rng.integers(150, 257)))
        out.append(k)
        left -= k
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--seeds", type=int, default=10)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    args = ap.parse_args()
    import torch
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
    from oracle import nn_ref_torch
    from test_bench_shape_gpu import _segmented_forward

    doc = {"oracle": "oracle/nn_ref_torch.py float64 on cuda", "weights": "random_weights(desc, 7921)",
           "device": torch.cuda.get_device_name(0), "configs": {}}
    for name in args.configs.split(","):
        cfg, precision, n = CONFIGS[name]
        desc = BASELINE_CONFIGS[cfg]["desc"]
        w = random_weights(desc, 7921)
        net = HipNet(desc, 0, precision)
        net.set_weights(to_blob(w))
        rows = []
        t0 = time.time()
        for seed in range(args.seeds):
            rng = np.random.default_rng(1000 + seed)
            x = random_planes(desc, n, 20251200 + 37 * cfg + seed)
            sizes = segments(n, rng)
            net.set_output_logits(False)
            got = _segmented_forward(net, desc, x, sizes)
            net.set_output_logits(True)
            got_l = _segmented_forward(net, desc, x, sizes)
            ref_l = nn_ref_torch.forward(desc, w, x, logits=True, device="cuda")
            ref = nn_ref_torch.forward(desc, w, x, device="cuda")
            rec = {"seed": seed, "rows": n, "segments": sizes, "outputs": []}
            for i, (g, r, gl, rl) in enumerate(zip(got, ref, got_l, ref_l)):
                d = np.abs(g.astype(np.float64) - r.astype(np.float64))
                rr = np.clip(r.astype(np.float64), 1e-30, None)
                gg = np.clip(g.astype(np.float64), 1e-30, None)
                kl = float((rr * np.log(rr / gg)).sum(axis=1).max())
                scale = max(1.0, float(np.abs(rl).max()))
                dl = np.abs(gl.astype(np.float64) - rl)
                rec["outputs"].append({"max": float(d.max()), "mean": float(d.mean()), "kl": kl,
                                       "logits_max": float(dl.max()), "logits_scale": scale,
                                       "logits_rel": float(dl.max()) / scale,
                                       "finite": bool(np.all(np.isfinite(g)))})
            rows.append(rec)
            print("%s seed %d: max %.3g mean %.3g kl %.3g logits_rel %.3g" % (
                name, seed, max(o["max"] for o in rec["outputs"]), max(o["mean"] for o in rec["outputs"]),
                max(o["kl"] for o in rec["outputs"]), max(o["logits_rel"] for o in rec["outputs"])), flush=True)
        net.close()
        summ = {k: max(max(o[k] for o in r["outputs"]) for r in rows) for k in ("max", "mean", "kl", "logits_rel")}
        doc["configs"][name] = {"baseline_config": cfg, "precision": "bf16x3 split" if precision == "fp32" else precision,
                                "net": "%dx%d" % (desc.residual_layers, desc.cnn_filter_size),
                                "seeds": rows, "max_over_seeds": summ, "seconds": time.time() - t0}
        print("%s max over %d seeds: %s" % (name, args.seeds, summ), flush=True)
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
