"""Import of the reference's Keras model files.

``desc_from_keras_json`` reads a ``data/<game>/models/<gen>.json`` document (the Keras
``model.to_json()`` the reference's manager writes, ``manager.py:113-127``) and returns the
:class:`NetDesc` of the residual net ``get_network_model`` builds (``model.py:154-296``), v1 or v2.
Both generations of v1 files are recognised:

* current ``model.py`` naming: ``initial-conv_conv2d`` / ``_bn``, ``ResLayer_<i>_conv0..bn1``,
  ``to_flatten_policy_head_<r>_conv2d`` / ``_bn``, ``value_flatten_conv2d`` (no BN), ``value_hidden``,
  ``value`` (softmax), Conv2D without bias;
* legacy files (keras 2.1.3-2.1.5, e.g. ``breakthrough/models/x6_102.json``): ``initial_conv2d`` with
  bias, ``to_flatten_value_head_conv2d`` + ``_bn``, ``value_hidden_layer``, sigmoid ``value`` -> the
  ``conv_bias`` / ``value_bn`` / ``value_sigmoid`` flags.

v2 files (``model.py:78-151``): ``ResLayer_<i>_bn_1 / conv1 / bn_2 / conv2`` pre-activation blocks,
optional ``ResLayer_<i>_se_compress / se_gating`` squeeze-excite Dense layers, a 1x1 ``initial-conv``
(bare in older files, ``initial-conv_conv2d / _bn`` in current ones) and the global-pooling value head
(``value_average`` + ``value_flatten_conv2d`` [+ ``_bn``], concatenated GAP-first, ``model.py:262-271``).
Files built by older model.py revisions with layers the current one cannot produce
(AveragePooling2D / Lambda reward heads, e.g. ``hexLG13/models/h1_229.json``) raise
:class:`NotSupported`.  The ``concat_all_layers`` value head (``model.py:251-260``: one
``value_flatten_<j>_conv2d`` + ``_bn`` per trunk layer, flattened and concatenated in layer order, e.g.
``hex19/models/h2_477.json``) maps to ``concat_all_layers``.

``weights_from_keras`` maps per-layer Keras weight lists (``layer.get_weights()``: Conv2D
``[kernel HWIO, bias?]``, BatchNormalization ``[gamma, beta, moving_mean, moving_variance]``, Dense
``[kernel, bias]``) onto the canonical blob order of ``desc.weight_spec`` - what a converter that
reads the reference's ``.h5`` with h5py (absent from this image) hands over.
"""
import json
import re

import numpy as np

from .desc import NetDesc, weight_spec

UNSUPPORTED_LAYERS = {"AveragePooling2D": "pooled reward head (not produced by model.py:154-296)",
                      "Lambda": "custom Lambda layer"}


class NotSupported(Exception):
    pass


def _layers(doc):
    if isinstance(doc, str):
        with open(doc) as f:
            doc = json.load(f)
    return doc, doc["config"]["layers"]


def _inbound(layer):
    nodes = layer.get("inbound_nodes") or []
    return [n[0] for n in nodes[0]] if nodes else []


def _is_conv(role):
    return re.match(r"(initial_conv|res\d+_conv[012]|policy\d+_conv|value\d*_conv)$", role) is not None


def _is_bn(role):
    return re.match(r"(initial_bn|res\d+_bn[012]|policy\d+_bn|value\d*_bn)$", role) is not None


def _is_se(role):
    return re.match(r"res\d+_se_(compress|gating)$", role) is not None


def roles(doc):
    """Maps every weight-carrying layer name of a model file to its role in weight_spec:
    ('initial_conv' | 'res<i>_conv<j>' | 'policy<r>_conv' | 'value_conv' | <same>_bn | 'res<i>_bn<j>'
    (v2 pre-activation) | 'res<i>_se_compress' | 'res<i>_se_gating' | 'policy<r>_dense' | 'value_hidden'
    | 'value_dense')."""
    doc, layers = _layers(doc)
    by_name = {l["name"]: l for l in layers}
    out = {}
    inp = [l["name"] for l in layers if l["class_name"] == "InputLayer"]
    for l in layers:
        n, cls = l["name"], l["class_name"]
        if cls == "Conv2D":
            m = re.match(r"ResLayer_(\d+)_conv([012])$", n)
            if m:
                out[n] = "res%s_conv%s" % m.groups()
            elif _inbound(l) == inp:
                out[n] = "initial_conv"
            elif re.search(r"policy_head_(\d+)", n):
                out[n] = "policy%s_conv" % re.search(r"policy_head_(\d+)", n).group(1)
            elif re.match(r"value_flatten_(\d+)_conv2d$", n):   # concat_all_layers, model.py:255-257
                out[n] = "value%s_conv" % re.match(r"value_flatten_(\d+)_conv2d$", n).group(1)
            elif "value" in n:
                out[n] = "value_conv"
            else:
                raise NotSupported("unrecognised Conv2D %s" % n)
        elif cls == "Dense":
            m = re.match(r"policy_(\d+)$", n)
            if m:
                out[n] = "policy%s_dense" % m.group(1)
            elif n.startswith("value_hidden"):
                out[n] = "value_hidden"
            elif n == "value":
                out[n] = "value_dense"
            elif re.match(r"ResLayer_(\d+)_se_(compress|gating)$", n):
                i, kind = re.match(r"ResLayer_(\d+)_se_(compress|gating)$", n).groups()
                out[n] = "res%s_se_%s" % (i, kind)
            else:
                raise NotSupported("unrecognised Dense %s" % n)
    for l in layers:
        if l["class_name"] == "BatchNormalization":
            m = re.match(r"ResLayer_(\d+)_bn_([12])$", l["name"])
            if m:                   # v2 pre-activation BN (its input is the stream or conv1)
                out[l["name"]] = "res%s_bn%s" % m.groups()
                continue
            src = _inbound(l)
            if len(src) != 1 or src[0] not in out or by_name[src[0]]["class_name"] != "Conv2D":
                raise NotSupported("BatchNormalization %s not after a conv" % l["name"])
            out[l["name"]] = out[src[0]].replace("conv", "bn")
    return out


def desc_from_keras_json(doc):
    """NetDesc of a v1 or v2 model file; NotSupported for other topologies."""
    doc, layers = _layers(doc)
    for l in layers:
        if l["class_name"] in UNSUPPORTED_LAYERS:
            raise NotSupported("%s: %s" % (l["class_name"], UNSUPPORTED_LAYERS[l["class_name"]]))
    r = roles(doc)
    cfg = {l["name"]: l["config"] for l in layers}
    cls = {l["name"]: l["class_name"] for l in layers}
    by_name = {l["name"]: l for l in layers}
    inp = next(l for l in layers if l["class_name"] == "InputLayer")
    shape = inp["config"]["batch_input_shape"]
    conv0 = next(n for n, v in r.items() if v == "initial_conv")
    if cfg[conv0].get("data_format", "channels_first") != "channels_first":
        raise NotSupported("channels_last input")
    C, H, W = shape[1], shape[2], shape[3]
    F = cfg[conv0]["filters"]
    v2 = any(re.match(r"ResLayer_\d+_(bn_[12]|conv2)$", n) for n in r)
    res_convs = [n for n, v in r.items() if re.match(r"res\d+_conv", v)]
    k = cfg[res_convs[0]]["kernel_size"][0] if res_convs else cfg[conv0]["kernel_size"][0]
    k0 = cfg[conv0]["kernel_size"][0]
    if k0 not in (1, 3) or cfg[conv0]["kernel_size"][1] != k0:
        raise NotSupported("initial conv kernel %s" % (cfg[conv0]["kernel_size"],))
    default_k0 = 1 if v2 else k
    blocks = sorted({int(v[3:v.index("_")]) for v in r.values() if v.startswith("res")})
    if blocks != list(range(len(blocks))):
        raise NotSupported("residual blocks are not numbered 0..B-1")
    npol = sorted(int(re.match(r"policy(\d+)_dense", v).group(1)) for v in r.values() if v.endswith("_dense")
                  and v.startswith("policy"))
    P = [cfg[next(n for n, v in r.items() if v == "policy%d_dense" % i)]["units"] for i in npol]
    hidden = next(n for n, v in r.items() if v == "value_hidden")
    value = next(n for n, v in r.items() if v == "value_dense")
    acts = {c.get("activation") for n, c in cfg.items() if cls[n] == "Activation"}
    leaky = any(cls[n] == "LeakyReLU" for n in cfg)
    if leaky and acts - {None}:
        raise NotSupported("mixed activations")
    if not leaky and acts != {"relu"}:
        raise NotSupported("activation %s" % sorted(a for a in acts if a))
    conv_bias = {bool(cfg[n].get("use_bias", False)) for n, v in r.items() if _is_conv(v)}
    if len(conv_bias) != 1:
        raise NotSupported("mixed use_bias across convs")
    eps = {cfg[n]["epsilon"] for n, v in r.items() if _is_bn(v)}
    if eps != {0.001}:
        raise NotSupported("BatchNormalization epsilon %s" % sorted(eps))
    # squeeze-excite (model.py:101-126): Dense(S, relu, no bias) -> Dense(F, sigmoid, no bias)
    se = {cfg[n]["units"] for n, v in r.items() if v.endswith("_se_compress")}
    if len(se) > 1:
        raise NotSupported("squeeze-excite units differ between blocks")
    for n, v in r.items():
        if _is_se(v):
            want = "relu" if v.endswith("compress") else "sigmoid"
            if cfg[n].get("use_bias") or cfg[n].get("activation") != want:
                raise NotSupported("squeeze-excite layer %s is not Dense(%s, no bias)" % (n, want))
    n_se = sum(1 for v in r.values() if v.endswith("_se_compress"))
    if n_se not in (0, len(blocks)):
        raise NotSupported("squeeze-excite on some blocks only")
    # global-pooling value head (model.py:262-271): Concatenate([GAP(trunk), flatten(value conv)])
    gap = False
    concat = False
    for n in cfg:
        if cls[n] == "GlobalAveragePooling2D" and not n.startswith("ResLayer_"):
            gap = True
        if cls[n] == "Concatenate":
            srcs = _inbound(by_name[n])

            def origin(x):
                while cls[x] in ("Flatten", "Reshape", "Activation", "BatchNormalization", "Dropout"):
                    x = _inbound(by_name[x])[0]
                return cls[x]
            origins = [origin(x) for x in srcs]
            if origins == ["GlobalAveragePooling2D", "Conv2D"]:
                continue
            if not v2 or set(origins) != {"Conv2D"}:
                raise NotSupported("concatenated value head %s" % n)
            # concat_all_layers (model.py:251-260): value conv j reads trunk layer j -- the initial
            # conv block's output, then each residual block's add -- in concatenation order

            def conv_of(x):
                while cls[x] != "Conv2D":
                    x = _inbound(by_name[x])[0]
                return x
            convs = [conv_of(x) for x in srcs]
            if [r.get(c) for c in convs] != ["value%d_conv" % j for j in range(len(blocks) + 1)]:
                raise NotSupported("concat_all_layers value convs out of layer order")
            for j, c in enumerate(convs):
                src = _inbound(by_name[c])[0]
                want = (lambda x: x.startswith("initial-conv") or r.get(x) == "initial_conv") if j == 0 else \
                    (lambda x, j=j: x == "ResLayer_%d_add" % (j - 1))
                if not want(src):
                    raise NotSupported("concat_all_layers value conv %d reads %s" % (j, src))
            concat = True
    flat = [c for n, c in cfg.items() if cls[n] == "Flatten"]
    dfs = {c.get("data_format") for c in flat}
    if len(dfs) != 1:
        raise NotSupported("mixed Flatten data_format")
    # Keras >= 2.1.6 Flatten(data_format='channels_first') permutes to (H, W, C); without the
    # argument (older files) or with channels_last it flattens the stored (C, H, W) order
    flatten_nchw = dfs.pop() != "channels_first"
    vact = cfg[value]["activation"]
    if vact not in ("softmax", "sigmoid"):
        raise NotSupported("value activation %s" % vact)
    return NetDesc(input_channels=C, input_columns=H, input_rows=W, cnn_filter_size=F, residual_layers=len(blocks),
                   policy_dist_count=P, value_hidden_size=cfg[hidden]["units"], num_values=cfg[value]["units"],
                   cnn_kernel_size=k, leaky_relu=leaky, flatten_nchw=flatten_nchw, conv_bias=conv_bias.pop(),
                   value_bn="value_bn" in r.values(), value_sigmoid=vact == "sigmoid",
                   resnet_v2=v2, initial_bn="initial_bn" in r.values(), se_units=se.pop() if se else 0,
                   global_pooling_value=gap, initial_kernel_size=0 if k0 == default_k0 else k0,
                   concat_all_layers=concat)


def weights_from_keras(doc, layer_weights):
    """layer_weights: {keras layer name: [arrays as layer.get_weights() returns them]} ->
    [(name, float32 array)] in weight_spec order (the blob gz_net_set_weights consumes)."""
    desc = desc_from_keras_json(doc)
    by_role = {}
    for name, role in roles(doc).items():
        ws = [np.asarray(a, dtype=np.float32) for a in layer_weights[name]]
        if _is_bn(role):
            g, b, m, v = ws
            by_role.update({role + "_gamma": g, role + "_beta": b, role + "_mean": m, role + "_var": v})
        elif _is_conv(role):
            by_role[role] = ws[0]
            if desc.conv_bias:
                by_role[role + "_bias"] = ws[1]
        elif _is_se(role):
            by_role[role] = ws[0]
        elif role.startswith("policy"):
            by_role[role] = ws[0]
            by_role[role.replace("_dense", "_bias")] = ws[1]
        elif role == "value_hidden":
            by_role["value_hidden"], by_role["value_hidden_bias"] = ws
        elif role == "value_dense":
            by_role["value_dense"], by_role["value_bias"] = ws
    out = []
    for name, shape in weight_spec(desc):
        a = by_role[name]
        if tuple(a.shape) != tuple(shape):
            raise ValueError("%s: shape %s, expected %s" % (name, a.shape, shape))
        out.append((name, a))
    return desc, out


def keras_layer_shapes(doc):
    """{layer name: [weight shapes]} a model file's layers carry (for converters / tests)."""
    desc = desc_from_keras_json(doc)
    spec = dict(weight_spec(desc))
    out = {}
    for name, role in roles(doc).items():
        if _is_bn(role):
            out[name] = [spec[role + s] for s in ("_gamma", "_beta", "_mean", "_var")]
        elif _is_conv(role):
            out[name] = [spec[role]] + ([spec[role + "_bias"]] if desc.conv_bias else [])
        elif _is_se(role):
            out[name] = [spec[role]]
        elif role.startswith("policy"):
            out[name] = [spec[role], spec[role.replace("_dense", "_bias")]]
        elif role == "value_hidden":
            out[name] = [spec["value_hidden"], spec["value_hidden_bias"]]
        else:
            out[name] = [spec["value_dense"], spec["value_bias"]]
    return out


def load_layer_weights_npz(path):
    """Per-layer weights saved as an .npz with keys '<layer name>/<index>' (what a converter reading
    the reference's .h5 with h5py writes: one array per entry of layer.get_weights())."""
    out = {}
    with np.load(path, allow_pickle=False) as z:
        for key in z.files:
            layer, idx = key.rsplit("/", 1)
            out.setdefault(layer, {})[int(idx)] = z[key]
    return {k: [v[i] for i in sorted(v)] for k, v in out.items()}
