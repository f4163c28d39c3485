"""Errors of the forward against the float64 oracle on boards of more than 64 positions, both
arithmetic modes: the 19 x 19 nets of tests/test_nn_19x19_gpu.py, the reference's v2 model files
beyond 8 x 8 and the reference templates on hexLG13 / amazons (tests/test_nn_v2_gpu.py,
tests/test_nn_gpu.py::test_template_geometries), so the tests' tolerances can be stated as ~3x
the worst measured.  Also times one 19 x 19 launch.  Usage: python tools/large_board_errors.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import NetDesc  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402
from oracle import nn_ref  # noqa: E402


def errs(got, ref):
    out = []
    for g, r in zip(got, ref):
        d = np.abs(g.astype(np.float64) - r)
        rr = np.clip(r, 1e-30, None)
        gg = np.clip(g.astype(np.float64), 1e-30, None)
        kl = float((rr * np.log(rr / gg)).sum(axis=1).max())
        out.append((float(d.max()), float(d.mean()), kl))
    return out


def run(tag, desc, w, xs, precisions=("bf16", "fp32")):
    for prec in precisions:
        try:
            net = HipNet(desc, 0, prec)
        except RuntimeError as e:
            print("%-28s %-4s unsupported: %s" % (tag, prec, e), flush=True)
            continue
        net.set_weights(to_blob(w))
        worst = [0.0, 0.0, 0.0]
        for x in xs:
            for e in errs(net.forward(x), nn_ref.forward(desc, w, x)):
                worst = [max(a, b) for a, b in zip(worst, e)]
        print("%-28s %-4s max %.3g mean %.3g kl %.3g" % (tag, prec, *worst), flush=True)
        net.close()


def main():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_nn_19x19_gpu as T19
    for name, desc in sorted(T19.NETS.items()):
        w = random_weights(desc, 7919, bias_std=0.2, res_gamma=T19.RES_GAMMA)
        run("19x19 " + name, desc, w, [random_planes(desc, n, 200 + n) for n in (1, 13)])
    with open(os.path.join(ROOT, "tests", "golden", "keras_descs.json")) as f:
        files = {k: NetDesc(**v["desc"]) for k, v in json.load(f).items() if "desc" in v and v["desc"]["resnet_v2"]}
    for k, desc in sorted(files.items()):
        w = random_weights(desc, 7919, bias_std=0.2, res_gamma=0.3)
        run("v2file " + k, desc, w, [random_planes(desc, n, 100 + n) for n in (1, 19)])
    # initial-conv widths: a 3x3 initial conv over C planes has K0 = 9 C rounded up to 32
    for C in (3, 5, 9, 12, 15, 24):
        for hw in (8, 13):
            desc = NetDesc(C, hw, hw, 64, 1, [hw * hw + 1, hw * hw + 1])
            run("k0 C=%d %dx%d" % (C, hw, hw), desc, random_weights(desc, 7919, bias_std=0.2),
                [random_planes(desc, 7, 100)])
    from test_nn_gpu import _template_desc
    for game in ("hexLG13", "amazons_10x10"):
        for hint in ("small", "medium", "large"):
            desc = _template_desc(game, hint)
            w = random_weights(desc, 7919, bias_std=0.2, res_gamma=0.15 if desc.residual_layers > 6 else 1.0)
            run("geom %s/%s" % (game, hint), desc, w, [random_planes(desc, 9, 31)], ("fp32",))
    # F = 256 on 8 x 8 in split precision (the two-pass kernel)
    desc = NetDesc(5, 8, 8, 256, 2, [155, 155])
    run("f256_8x8", desc, random_weights(desc, 7919, bias_std=0.2), [random_planes(desc, n, 100 + n) for n in (1, 7)],
        ("fp32",))
    # timing: the hex19 net, 1,024 rows
    desc = T19.H2_477
    w = to_blob(random_weights(desc, 7921, res_gamma=T19.RES_GAMMA))
    x = random_planes(desc, 1024, 5)
    for prec in ("bf16", "fp32"):
        net = HipNet(desc, 0, prec)
        net.set_weights(w)
        net.forward(x)
        t0 = time.time()
        for _ in range(3):
            net.forward(x)
        ms = net.last_kernel_ms()
        print("hex19 h2_477 %s 1,024 rows: kernel %.2f ms, %.1f TFLOP/s algorithmic (wall %.1f ms per forward)"
              % (prec, ms, desc.flops_per_eval() * 1024 / (ms * 1e-3) / 1e12, (time.time() - t0) / 3 * 1e3), flush=True)
        net.close()


if __name__ == "__main__":
    main()
