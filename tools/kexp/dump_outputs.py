"""Writes the cfg2 split forward's outputs on fixed inputs to an .npz (kernel experiments: two
processes with different GZ_LIB_DIR builds, then compare.py).  usage: dump_outputs.py OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from galvanise_zero_amd._native import HipNet  # noqa: E402
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS  # noqa: E402
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob  # noqa: E402

desc = BASELINE_CONFIGS[2]["desc"]
net = HipNet(desc, 0, "fp32")
net.set_weights(to_blob(random_weights(desc, 7921)))
out = {}
for n in (1, 300, 1031):
    for i, o in enumerate(net.forward(random_planes(desc, n, 17 + n))):
        out["n%d_out%d" % (n, i)] = o
np.savez(sys.argv[1], **out)
