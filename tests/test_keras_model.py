"""Import of the reference's Keras model files (galvanise_zero_amd/nn/keras_model.py):
the v1 files parse to the NetDesc recorded in tests/golden/keras_v1_descs.json (shapes checked
against SURVEY appendix A), the others are rejected with the reason; per-layer Keras weights map
onto the blob so that the oracle forward of the mapped blob equals a forward computed directly
from the Keras-named layers."""
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd.nn import keras_model as K
from galvanise_zero_amd.nn.desc import NetDesc
from oracle import nn_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "keras_v1_descs.json")
REF = "/root/reference/data"


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_golden_v1_files(golden):
    ok = {k: NetDesc(**v["desc"]) for k, v in golden.items() if "desc" in v}
    assert set(ok) == {"amazons_10x10/models/h1_27.json", "breakthrough/models/x6_102.json",
                       "breakthrough/models/x6_111.json", "breakthroughSmall/models/x1_132.json",
                       "breakthroughSmall/models/x1_42.json"}
    d = ok["breakthrough/models/x6_102.json"]      # 10x128, 5x8x8, 155/155, hidden 256
    assert (d.input_channels, d.input_columns, d.input_rows, d.cnn_filter_size, d.residual_layers) == (5, 8, 8, 128, 10)
    assert d.policy_dist_count == [155, 155] and d.value_hidden_size == 256 and d.num_values == 2
    assert d.conv_bias and d.value_bn and d.value_sigmoid and d.flatten_nchw
    assert ok["amazons_10x10/models/h1_27.json"].policy_dist_count == [3041, 3041]
    rejected = {k: v["not_supported"] for k, v in golden.items() if "not_supported" in v}
    assert "GlobalAveragePooling2D" in rejected["breakthrough/models/f1_396.json"]
    assert len(rejected) + len(ok) == len(golden)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")
def test_importer_matches_golden(golden):
    import dataclasses
    for key, v in golden.items():
        path = os.path.join(REF, key)
        if "desc" in v:
            assert dataclasses.asdict(K.desc_from_keras_json(path)) == v["desc"], key
        else:
            with pytest.raises(K.NotSupported):
                K.desc_from_keras_json(path)


def _keras_forward(desc, lw, names, x):
    """Forward written directly against the Keras layer names (conv + bias -> BN -> relu ...)."""
    def conv(t, name):
        k, b = lw[name][0].astype(np.float64), lw[name][1]
        return nn_ref._conv_same(t, k) + b

    def bn(t, name):
        g, be, m, v = (a.astype(np.float64) for a in lw[name])
        return g * (t - m) / np.sqrt(v + 1e-3) + be

    relu = lambda t: np.maximum(t, 0)   # noqa: E731
    t = np.transpose(x.astype(np.float64), (0, 2, 3, 1))
    t = relu(bn(conv(t, names["initial_conv"]), names["initial_bn"]))
    for i in range(desc.residual_layers):
        y = relu(bn(conv(t, names["res%d_conv0" % i]), names["res%d_bn0" % i]))
        y = bn(conv(y, names["res%d_conv1" % i]), names["res%d_bn1" % i])
        t = relu(t + y)
    flat = lambda a: np.transpose(a, (0, 3, 1, 2)).reshape(a.shape[0], -1)   # noqa: E731  (C,H,W)
    outs = []
    for r in range(desc.role_count):
        h = relu(bn(conv(t, names["policy%d_conv" % r]), names["policy%d_bn" % r]))
        z = flat(h) @ lw[names["policy%d_dense" % r]][0] + lw[names["policy%d_dense" % r]][1]
        outs.append(nn_ref._softmax(z))
    v = relu(bn(conv(t, names["value_conv"]), names["value_bn"]))
    hid = relu(flat(v) @ lw[names["value_hidden"]][0] + lw[names["value_hidden"]][1])
    outs.append(1 / (1 + np.exp(-(hid @ lw[names["value_dense"]][0] + lw[names["value_dense"]][1]))))
    return outs


def test_weight_mapping_x6_102(golden):
    from dataclasses import replace
    g = golden["breakthrough/models/x6_102.json"]
    desc = NetDesc(**g["desc"])
    rng = np.random.default_rng(5)
    lw = {}
    for name, shapes in g["layers"].items():
        arrs = []
        for j, s in enumerate(shapes):
            if len(g["layers"][name]) == 4 and j in (0, 3):           # BN gamma / variance
                arrs.append(rng.uniform(0.5, 1.5, size=s).astype(np.float32))
            else:
                arrs.append((rng.normal(0, 0.1, size=s) if len(s) == 1 else
                             rng.normal(0, np.sqrt(1.0 / np.prod(s[:-1])), size=s)).astype(np.float32))
        lw[name] = arrs
    doc = _doc_from_golden(g)
    d2, mapped = K.weights_from_keras(doc, lw)
    assert d2 == desc
    roles = K.roles(doc)
    names = {v: k for k, v in roles.items()}
    x = np.random.default_rng(1).integers(0, 2, size=(3, 5, 8, 8)).astype(np.float32)
    got = nn_ref.forward(desc, mapped, x)
    exp = _keras_forward(desc, lw, names, x)
    for a, b in zip(got, exp):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    assert replace(desc, residual_layers=0).residual_layers == 0


def _doc_from_golden(g):
    """A minimal Keras-JSON document with the golden file's layers (names, classes, configs the
    importer reads) - the reference file itself does not travel."""
    d = NetDesc(**g["desc"])
    layers = [{"class_name": "InputLayer", "name": "inputs_board", "inbound_nodes": [],
               "config": {"batch_input_shape": [None, d.input_channels, d.input_columns, d.input_rows]}}]

    def add(cls, name, src, **cfg):
        layers.append({"class_name": cls, "name": name, "config": cfg,
                       "inbound_nodes": [[[src, 0, 0, {}]]] if src else []})

    conv_cfg = dict(data_format="channels_first", kernel_size=[3, 3], use_bias=True)
    add("Conv2D", "initial_conv2d", "inputs_board", filters=d.cnn_filter_size, **conv_cfg)
    add("BatchNormalization", "initial_bn", "initial_conv2d", epsilon=0.001)
    add("Activation", "initial_act", "initial_bn", activation="relu")
    for i in range(d.residual_layers):
        add("Conv2D", "ResLayer_%d_conv0" % i, "x", filters=d.cnn_filter_size, **conv_cfg)
        add("BatchNormalization", "ResLayer_%d_bn0" % i, "ResLayer_%d_conv0" % i, epsilon=0.001)
        add("Conv2D", "ResLayer_%d_conv1" % i, "x", filters=d.cnn_filter_size, **conv_cfg)
        add("BatchNormalization", "ResLayer_%d_bn1" % i, "ResLayer_%d_conv1" % i, epsilon=0.001)
    for r, p in enumerate(d.policy_dist_count):
        add("Conv2D", "to_flatten_policy_head_%d_conv2d" % r, "x", filters=2, **dict(conv_cfg, kernel_size=[1, 1]))
        add("BatchNormalization", "to_flatten_policy_head_%d_bn" % r, "to_flatten_policy_head_%d_conv2d" % r,
            epsilon=0.001)
        add("Flatten", "flatten_p%d" % r, "x")
        add("Dense", "policy_%d" % r, "x", units=p, activation="softmax")
    add("Conv2D", "to_flatten_value_head_conv2d", "x", filters=1, **dict(conv_cfg, kernel_size=[1, 1]))
    add("BatchNormalization", "to_flatten_value_head_bn", "to_flatten_value_head_conv2d", epsilon=0.001)
    add("Flatten", "flatten_v", "x")
    add("Dense", "value_hidden_layer", "x", units=d.value_hidden_size, activation="relu")
    add("Dense", "value", "x", units=d.num_values, activation="sigmoid")
    assert set(l["name"] for l in layers if l["class_name"] in ("Conv2D", "BatchNormalization", "Dense")) == \
        set(g["layers"])
    return {"class_name": "Model", "config": {"layers": layers}}


def test_layer_weights_npz_roundtrip(tmp_path, golden):
    g = golden["breakthroughSmall/models/x1_42.json"]
    rng = np.random.default_rng(2)
    lw = {n: [rng.normal(size=s).astype(np.float32) for s in shapes] for n, shapes in g["layers"].items()}
    path = str(tmp_path / "w.npz")
    np.savez(path, **{"%s/%d" % (n, i): a for n, arrs in lw.items() for i, a in enumerate(arrs)})
    back = K.load_layer_weights_npz(path)
    assert set(back) == set(lw)
    for n in lw:
        assert all(np.array_equal(a, b) for a, b in zip(lw[n], back[n]))
