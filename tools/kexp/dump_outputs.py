"""Writes a config's split forward outputs on fixed inputs to an .npz (kernel experiments: two
processes with different GZ_LIB_DIR builds, then compare).  usage: dump_outputs.py OUT.npz [CFG]
(default cfg2)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402

cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
desc = BASELINE_CONFIGS[cfg]["desc"]
net = HipNet(desc, 0, "fp32")
net.set_weights(to_blob(random_weights(desc, 7921)))
out = {}
for n in ((1, 300, 1031) if cfg == 2 else (1, 300)):
    for i, o in enumerate(net.forward(random_planes(desc, n, 17 + n))):
        out["n%d_out%d" % (n, i)] = o
np.savez(sys.argv[1], **out)
