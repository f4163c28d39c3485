"""Max |difference| of every output between two kernel variants (GZ_KERNEL_VARIANT) on cfg2-shaped
nets of 0 / 1 / 6 residual blocks, at a few launch sizes.  Usage: python tools/variant_diff.py 21 23"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import NetDesc  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402

va, vb = sys.argv[1], sys.argv[2]
for blocks in (0, 1, 6):
    desc = NetDesc(12, 8, 8, 128, blocks, [155, 155])
    w = to_blob(random_weights(desc, 5, bias_std=0.2))
    for n in (2, 33, 512):
        x = random_planes(desc, n, 4)
        outs = []
        for v in (va, vb):
            os.environ["GZ_KERNEL_VARIANT"] = v
            net = HipNet(desc, 0, "fp32")
            net.set_weights(w)
            outs.append(net.forward(x))
        d = [float(np.max(np.abs(a - b))) for a, b in zip(*outs)]
        rows = [int(np.argmax(np.max(np.abs(a - b).reshape(n, -1), axis=1))) for a, b in zip(*outs)]
        print("blocks %d rows %4d max|d| per output %s worst rows %s" % (blocks, n, ["%.3g" % e for e in d], rows), flush=True)
