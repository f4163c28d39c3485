"""CPU tests pinning the NN oracle (oracle/nn_ref.py).

No reference test holds a numeric NN output and the trained .h5 weights are absent, so
the numpy oracle is pinned two ways: (1) against an independent torch-CPU float64 implementation of
the same Keras layer semantics (conv2d 'same', inference BatchNormalization eps=1e-3, Flatten order),
and (2) against committed golden vectors (tests/golden/nn_*.npz, made by tests/golden/make_nn_golden.py)
that freeze its output.  Shapes/orderings are pinned by the reference model JSONs (see test_arch).
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as tF

from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS, NetDesc, blob_size, weight_spec
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob, from_blob
from oracle import nn_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def torch_forward(desc, weights, planes):
    w = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights}
    act = (lambda t: tF.leaky_relu(t, 0.03)) if desc.leaky_relu else tF.relu
    x = torch.tensor(planes, dtype=torch.float64)

    def conv(t, name):
        k = w[name] if isinstance(name, str) else name
        b = w.get(name + "_bias") if isinstance(name, str) and desc.conv_bias else None
        return tF.conv2d(t, k.permute(3, 2, 0, 1), bias=b, padding=k.shape[0] // 2)

    def bn(t, p):
        return tF.batch_norm(t, w[p + "_mean"], w[p + "_var"], w[p + "_gamma"], w[p + "_beta"],
                             training=False, eps=1e-3)

    x = act(bn(conv(x, "initial_conv"), "initial_bn"))
    for i in range(desc.residual_layers):
        y = act(bn(conv(x, "res%d_conv0" % i), "res%d_bn0" % i))
        y = bn(conv(y, "res%d_conv1" % i), "res%d_bn1" % i)
        x = act(x + y)

    def flat(t):
        if not desc.flatten_nchw:
            t = t.permute(0, 2, 3, 1)
        return t.reshape(t.shape[0], -1)

    outs = []
    for r in range(desc.role_count):
        h = act(bn(conv(x, "policy%d_conv" % r), "policy%d_bn" % r))
        z = flat(h) @ w["policy%d_dense" % r] + w["policy%d_bias" % r]
        outs.append(torch.softmax(z, 1).numpy())
    v = conv(x, "value_conv")
    if desc.value_bn:
        v = bn(v, "value_bn")
    v = act(v)
    hid = act(flat(v) @ w["value_hidden"] + w["value_hidden_bias"])
    z = hid @ w["value_dense"] + w["value_bias"]
    outs.append((torch.sigmoid(z) if desc.value_sigmoid else torch.softmax(z, 1)).numpy())
    return outs


VARIANTS = [
    NetDesc(5, 6, 6, 64, 2, [81, 81]),
    NetDesc(5, 8, 8, 128, 2, [155, 155]),
    NetDesc(5, 8, 8, 64, 1, [65, 65], num_values=3, leaky_relu=True),
    NetDesc(5, 6, 6, 64, 1, [81, 81], flatten_nchw=True),
    # legacy v1 model file semantics (x6_102.json): conv biases, value BN, sigmoid value
    NetDesc(5, 8, 8, 64, 2, [155, 155], flatten_nchw=True, conv_bias=True, value_bn=True, value_sigmoid=True),
]


@pytest.mark.parametrize("desc", VARIANTS)
def test_oracle_matches_torch(desc):
    w = random_weights(desc, 11, bias_std=0.2)
    x = random_planes(desc, 9, 3)
    a = nn_ref.forward(desc, w, x)
    b = torch_forward(desc, w, x)
    assert len(a) == desc.role_count + 1
    for u, v in zip(a, b):
        np.testing.assert_allclose(u, v, rtol=1e-5, atol=1e-6)
    for u in (a[:-1] if desc.value_sigmoid else a):   # sigmoid value outputs are independent
        np.testing.assert_allclose(u.sum(axis=1), 1.0, atol=1e-5)


def test_blob_roundtrip():
    d = BASELINE_CONFIGS[2]["desc"]
    w = random_weights(d, 5)
    blob = to_blob(w)
    assert blob.size == blob_size(d) == 1839688
    w2 = from_blob(d, blob)
    for (n1, a), (n2, b) in zip(w, w2):
        assert n1 == n2 and np.array_equal(a, b)


def test_flops_match_survey():
    # SURVEY 8(d) / BASELINE.md: MFLOP per leaf eval per config
    expect = {1: 10.89, 2: 227.42, 3: 378.37, 4: 4789.3, 5: 4726.9}
    for k, v in expect.items():
        assert abs(BASELINE_CONFIGS[k]["desc"].flops_per_eval() / 1e6 - v) < 0.01 * v


@pytest.mark.parametrize("name", ["nn_cfg1", "nn_cfg2"])
def test_oracle_golden(name):
    path = os.path.join(GOLDEN, name + ".npz")
    g = np.load(path)
    cfg = int(g["cfg"])
    desc = BASELINE_CONFIGS[cfg]["desc"]
    w = random_weights(desc, int(g["wseed"]), bias_std=float(g["bias_std"]))
    x = random_planes(desc, int(g["n"]), int(g["xseed"]))
    np.testing.assert_array_equal(x, g["planes"])
    out = nn_ref.forward(desc, w, x)
    for i, o in enumerate(out):
        np.testing.assert_allclose(o, g["out%d" % i], rtol=1e-6, atol=1e-7)


def test_arch_fixture_shapes():
    """Policy sizes / input shapes / BN epsilon agree with the reference model JSONs."""
    path = os.path.join(GOLDEN, "arch.json")
    arch = json.load(open(path))
    for game, info in arch.items():
        for k, v in BASELINE_CONFIGS.items():
            if v["game"] == game:
                d = v["desc"]
                assert info["input_shape"] == [d.input_channels, d.input_columns, d.input_rows]
                assert info["policy_units"] == d.policy_dist_count
                assert all(abs(e - 1e-3) < 1e-12 for e in info["bn_epsilon"])


@pytest.mark.parametrize("desc", VARIANTS)
def test_torch_cpu_fp32_matches_oracle(desc):
    """oracle/nn_torch.py (bench.py's CPU-baseline network, float32 torch-CPU) agrees with the
    float64 oracle to float32 accuracy."""
    from oracle.nn_torch import TorchCPUNet
    w = random_weights(desc, 3)
    x = random_planes(desc, 9, 4)
    for a, b in zip(TorchCPUNet(desc, w).predict_on_batch(x), nn_ref.forward(desc, w, x)):
        assert a.dtype == np.float32 and a.shape == b.shape
        assert float(np.abs(a - b).max()) < 2e-5


ORACLE_DESCS = {
    "v1": NetDesc(5, 8, 8, 32, 2, [17, 19], value_hidden_size=16),
    "v1_legacy_leaky": NetDesc(5, 6, 6, 16, 1, [9, 9], value_hidden_size=8, conv_bias=True, value_bn=True,
                               value_sigmoid=True, flatten_nchw=True, leaky_relu=True),
    "v2_se_gap": NetDesc(5, 7, 7, 24, 2, [11, 13], value_hidden_size=8, num_values=3, resnet_v2=True, se_units=9,
                         global_pooling_value=True, value_bn=True),
    "v2_concat": NetDesc(5, 7, 6, 16, 3, [11, 13], value_hidden_size=8, resnet_v2=True, concat_all_layers=True),
}


@pytest.mark.parametrize("name", list(ORACLE_DESCS))
def test_torch_f64_oracle_matches_numpy_oracle(name):
    """oracle/nn_ref_torch.py (float64 torch, the GPU-side oracle of tools/split_error_dist.py)
    restates oracle/nn_ref.forward: equal to ~1e-12 on the CPU, probabilities and logits."""
    from oracle import nn_ref_torch
    desc = ORACLE_DESCS[name]
    w = random_weights(desc, 3, bias_std=0.2)
    x = random_planes(desc, 7, 4)
    for logits in (False, True):
        a = nn_ref.forward(desc, w, x, logits=logits)
        b = nn_ref_torch.forward(desc, w, x, logits=logits)
        for u, v in zip(a, b):
            assert u.shape == v.shape
            assert np.abs(u.astype(np.float64) - v.astype(np.float64)).max() <= (1e-7 if not logits else 1e-10)


def test_concat_all_layers_value_head_semantics():
    """model.py:251-260: the value Dense reads (B + 1) HW features in layer order, layer j's block
    its own 1x1 conv + BN + act.  Wiring check: with layer j's rows of value_hidden zeroed, the value
    no longer depends on layer j's conv (and does on every other layer's)."""
    desc = ORACLE_DESCS["v2_concat"]
    spec = dict(weight_spec(desc))
    B, hw = desc.residual_layers, desc.hw
    assert spec["value_hidden"] == ((B + 1) * hw, desc.value_hidden_size)
    assert all("value%d_conv" % j in spec for j in range(B + 1)) and "value_conv" not in spec
    assert desc.flops_trunk() - NetDesc(**{**desc.__dict__, "concat_all_layers": False}).flops_trunk() == B * 2 * hw * 16
    w = random_weights(desc, 3)
    x = random_planes(desc, 5, 4)
    for j in range(B + 1):
        wz = [(k, a.copy()) for k, a in w]
        dict(wz)["value_hidden"][j * hw:(j + 1) * hw] = 0.0
        base = nn_ref.forward(desc, wz, x, logits=True)[-1]
        for jj in range(B + 1):
            wp = [(k, a * 1.7 if k == "value%d_conv" % jj else a) for k, a in wz]
            moved = not np.allclose(nn_ref.forward(desc, wp, x, logits=True)[-1], base, rtol=0, atol=1e-12)
            assert moved == (jj != j), (j, jj)
