"""Boards beyond 13 x 13 (up to 19 x 19): the reference's hex19 network (data/hex19/models/h2_477.json:
v2, 10 blocks x 80 filters with squeeze-excite, 15 planes, policies 362 / 363, the concat-all-layers
value head, model.py:78-151, 251-260) and v1 nets on 19 x 19, against the float64 oracle
(oracle/nn_ref.forward).

Kernels: trunk_kernel(_v2)<128, 23, 1, 1, P> -- one board per workgroup in a single LDS image of
padded 288-byte rows (107 KB), the residual stream in a device scratch, the looped conv; split
precision by two passes per conv (P = 2: the hi + lo image would need 201 KB).  Boards of 12 .. 22
position tiles run on the same 23-tile kernels (tiles off the board read the zero rows and store
nothing); nets of <= 64 filters are padded to the 128-filter kernels there.

Tolerances: ~3x the worst measured on MI355X for these nets and seeds (profiles/r05c_large_board_errors.log);
weights damped as in tests/test_nn_v2_gpu.py (res_gamma) so the softmaxes stay in the interior.
"""
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd.nn.desc import NetDesc
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
from oracle import nn_ref

pytestmark = pytest.mark.gpu

with open(os.path.join(os.path.dirname(__file__), "golden", "keras_descs.json")) as _f:
    H2_477 = NetDesc(**json.load(_f)["hex19/models/h2_477.json"]["desc"])

NETS = {
    # the reference's own 19 x 19 model file as the importer reads it
    "hex19_h2_477": H2_477,
    # v1 19 x 19, 128 filters, the plain value head (flatten NHWC)
    "v1_19x19_f128": NetDesc(5, 19, 19, 128, 3, [362, 362]),
    # v1 19 x 19 with 64 filters (run on the 128-filter kernels) and a 3-value head, flatten NCHW
    "v1_19x19_f64_v3": NetDesc(4, 19, 19, 64, 2, [361, 361], num_values=3, flatten_nchw=True, leaky_relu=True),
    # 15 x 15 (15 position tiles on the 23-tile kernel), v2 with squeeze-excite and a pooling value head
    "v2_15x15_gap": NetDesc(5, 15, 15, 96, 3, [226, 226], resnet_v2=True, se_units=32, global_pooling_value=True),
}
RES_GAMMA = 0.3

# (max |err|, mean |err|) vs the float64 oracle: 3 x the worst measured over these nets on MI355X
# (profiles/r05c_large_board_errors.log: bf16 8.8e-4 / 5.7e-4, split 1.8e-6 / 1.4e-6, KL 1.3e-7)
TOL = {
    "bf16": (2.7e-3, 1.8e-3),
    "bf16x3": (5.4e-6, 4.3e-6),
}
TOL_FP32_KL = 4e-7


def _err(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return float(d.max()), float(d.mean())


def _kl(ref, got):
    r = np.clip(ref.astype(np.float64), 1e-30, None)
    g = np.clip(got.astype(np.float64), 1e-30, None)
    return float((r * np.log(r / g)).sum(axis=1).max())


def _net(desc, w, device, precision):
    from galvanise_zero_amd._native import HipNet
    net = HipNet(desc, device, precision)
    net.set_weights(to_blob(w))
    return net


@pytest.mark.parametrize("precision", ["bf16", "bf16x3"])
@pytest.mark.parametrize("name", sorted(NETS))
def test_large_board_parity(name, precision, hip_device):
    desc = NETS[name]
    w = random_weights(desc, 7919, bias_std=0.2, res_gamma=RES_GAMMA)
    net = _net(desc, w, hip_device, precision)
    tol = TOL[precision]
    for n in (1, 13):
        x = random_planes(desc, n, 200 + n)
        got = net.forward(x)
        ref = nn_ref.forward(desc, w, x)
        for i, (g, r) in enumerate(zip(got, ref)):
            assert g.shape == r.shape and np.all(np.isfinite(g))
            er = _err(g, r)
            kl = _kl(r, g)
            print("%s %s n=%d out%d vs_ref max %.3g mean %.3g kl %.3g" % (name, precision, n, i, er[0], er[1], kl))
            assert er[0] <= tol[0] and er[1] <= tol[1], (name, precision, n, i, er)
            if precision == "bf16x3":
                assert kl <= TOL_FP32_KL, (name, n, i, kl)
    net.close()


@pytest.mark.parametrize("precision", ["bf16", "bf16x3"])
def test_large_board_batch_invariance(precision, hip_device):
    """Every row of the 19 x 19 hex19 net computes identically whatever the batch composition or
    slot (the basis of bit-exact PUCT under batching)."""
    desc = H2_477
    net = _net(desc, random_weights(desc, 3, bias_std=0.2, res_gamma=RES_GAMMA), hip_device, precision)
    x = random_planes(desc, 300, 9)
    full = net.forward(x)
    perm = np.random.default_rng(0).permutation(300)[:37]
    for a, b in zip(full, net.forward(x[perm])):
        assert np.array_equal(a[perm], b)
    for a, b in zip(full, net.forward(x[5:6])):
        assert np.array_equal(a[5:6], b)
    net.close()
