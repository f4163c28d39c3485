"""ORACLE (test infrastructure only) -- CPU restatement of the reference policy/value CNN forward.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (galvanise_zero_amd) never does.

Restates ``get_network_model`` (reference ``src/ggpzero/nn/model.py:154-296``, v1 / AG0 path) as
executed by Keras 2.2 / TF 1.12 ``predict_on_batch`` (``src/ggpzero/util/cppinterface.py:119``):

* ``conv2d_block``  model.py:25-44  -- Conv2D(use_bias=False, padding same) -> BatchNormalization
  (axis=1, inference: gamma*(x-mean)/sqrt(var+eps)+beta, eps=1e-3) -> activation
* ``residual_block_v1`` model.py:47-75 -- conv-BN-act-conv-BN, add(tensor, x), act
* policy heads model.py:223-241 -- conv1x1(2)+BN+act, Flatten, Dense(P_r) softmax
* value head model.py:273-291 -- conv1x1(1) do_bn=False + act, Flatten, Dense(hidden)+act,
  Dense(V) softmax
* Flatten: channels_first data in Keras >= 2.1.6 is permuted to (H, W, C) before flattening
  (``flatten_nchw=False``); legacy files flatten (C, H, W).
* Legacy v1 model files (data/breakthrough/models/x6_102.json, keras 2.1.3): Conv2D(use_bias=True)
  everywhere (``conv_bias``), BatchNormalization after the value head's conv (``value_bn``), value
  Dense with sigmoid (``value_sigmoid``).
* v2 (``resnet_v2``) model.py:78-151, 171-198: initial 1x1 ``conv2d_block`` (BN + act, or a bare conv
  in older files: ``initial_bn=False``), blocks BN-act-conv-BN-act-conv, squeeze-excite
  (``se_block`` :101-126: GlobalAveragePooling2D -> Dense(S, relu, no bias) -> Dense(F, sigmoid, no
  bias) -> multiply), add without activation (:147); dropout is the identity at inference.
* ``global_pooling_value`` model.py:262-271: value features = concat(GAP(trunk) [F], flatten(value
  1x1 conv + BN + act) [HW]).
* ``concat_all_layers`` model.py:251-260 (v2 only: ``all_layers`` is built by the v2 branch,
  :173-198): value features = concat over the trunk layers (initial conv block output, then each
  residual block's add) of flatten(1x1 conv(1) + BN + act) [HW each], in layer order.

Arithmetic is float64 (the fp32 TF result is within ~1e-6 of it); outputs are float32 like
``predict_on_batch``.  Parity of the reference NN itself is *unpinned*: no reference test holds a
numeric NN output and the trained weights are absent.
"""

import numpy as np

EPS = 1e-3
LEAKY = 0.03


def _act(x, leaky):
    if leaky:
        return np.where(x > 0, x, LEAKY * x)
    return np.maximum(x, 0.0)


def _bn(x, w, prefix):
    g, b, m, v = (w[prefix + s].astype(np.float64) for s in ("_gamma", "_beta", "_mean", "_var"))
    return g * (x - m) / np.sqrt(v + EPS) + b


def _conv_same(x, k):
    """x: [N, H, W, Cin] float64; k: [kh, kw, Cin, Cout] (Keras HWIO), 'same' padding, no bias."""
    kh, kw = k.shape[0], k.shape[1]
    ph, pw = kh // 2, kw // 2
    N, H, W, _ = x.shape
    xp = np.pad(x, ((0, 0), (ph, ph), (pw, pw), (0, 0)))
    out = np.zeros((N, H, W, k.shape[3]))
    for dy in range(kh):
        for dx in range(kw):
            out += xp[:, dy:dy + H, dx:dx + W, :] @ k[dy, dx].astype(np.float64)
    return out


def _softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def _flatten(x, nchw):
    # x: [N, H, W, C]
    if nchw:
        x = np.transpose(x, (0, 3, 1, 2))
    return x.reshape(x.shape[0], -1)


def _sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def _value_out(desc, z):
    return (_sigmoid(z) if getattr(desc, "value_sigmoid", False) else _softmax(z)).astype(np.float32)


def forward(desc, weights, planes, logits=False):
    """planes: float32 [N, C, H, W] (the poll() layout, cppinterface.py:114).

    Returns [policy_0 [N,P_0], ..., policy_{R-1}, value [N,V]] float32 (model.py:294 order);
    logits=True: the heads' pre-activation outputs (before the softmaxes / sigmoid), float64."""
    w = dict(weights)
    leaky = desc.leaky_relu
    logits_out = logits

    def conv(x, name):
        y = _conv_same(x, w[name])
        if getattr(desc, "conv_bias", False):
            y = y + w[name + "_bias"].astype(np.float64)
        return y

    x = np.transpose(planes.astype(np.float64), (0, 2, 3, 1))     # NHWC
    v2 = getattr(desc, "resnet_v2", False)
    x = conv(x, "initial_conv")
    if not v2 or desc.initial_bn:
        x = _act(_bn(x, w, "initial_bn"), leaky)
    layers = [x]                                                   # all_layers, model.py:181,198
    for i in range(desc.residual_layers):
        t = x
        if v2:
            y = conv(_act(_bn(x, w, "res%d_bn1" % i), leaky), "res%d_conv1" % i)
            y = conv(_act(_bn(y, w, "res%d_bn2" % i), leaky), "res%d_conv2" % i)
            if desc.se_units:
                m = y.mean(axis=(1, 2))                                               # [N, F]
                h = np.maximum(m @ w["res%d_se_compress" % i].astype(np.float64), 0.0)
                y = y * _sigmoid(h @ w["res%d_se_gating" % i].astype(np.float64))[:, None, None, :]
            x = t + y
        else:
            y = _act(_bn(conv(x, "res%d_conv0" % i), w, "res%d_bn0" % i), leaky)
            y = _bn(conv(y, "res%d_conv1" % i), w, "res%d_bn1" % i)
            x = _act(t + y, leaky)
        layers.append(x)
    outs = []
    for r in range(desc.role_count):
        h = _act(_bn(conv(x, "policy%d_conv" % r), w, "policy%d_bn" % r), leaky)
        logits_r = _flatten(h, desc.flatten_nchw) @ w["policy%d_dense" % r].astype(np.float64)
        logits_r = logits_r + w["policy%d_bias" % r]
        outs.append(logits_r if logits_out else _softmax(logits_r).astype(np.float32))
    if getattr(desc, "concat_all_layers", False):
        flat = np.concatenate([_flatten(_act(_bn(conv(l, "value%d_conv" % j), w, "value%d_bn" % j), leaky),
                                        desc.flatten_nchw) for j, l in enumerate(layers)], axis=1)
    else:
        v = conv(x, "value_conv")
        if getattr(desc, "value_bn", False):
            v = _bn(v, w, "value_bn")
        v = _act(v, leaky)
        flat = _flatten(v, desc.flatten_nchw)
        if getattr(desc, "global_pooling_value", False):
            flat = np.concatenate([x.mean(axis=(1, 2)), flat], axis=1)
    hid = _act(flat @ w["value_hidden"].astype(np.float64) + w["value_hidden_bias"], leaky)
    val = hid @ w["value_dense"].astype(np.float64) + w["value_bias"]
    outs.append(val if logits_out else _value_out(desc, val))
    return outs


# ---------------------------------------------------------------------------------------------
# bf16-emulating variant: same math as the HIP kernel's numerics contract (BN folded into the
# conv in float32, folded conv weights and conv *inputs* rounded to bf16 RNE, float accumulate,
# residual stream and heads in full precision).  Used to test the kernel tightly; the float64
# forward() above is the reference semantics the stated tolerance is measured against.

def bf16_round(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return (u.astype(np.uint32) << 16).view(np.float32)


def _fold(w, conv, bn):
    k = w[conv].astype(np.float32)
    g, b, m, v = (w[bn + s].astype(np.float32) for s in ("_gamma", "_beta", "_mean", "_var"))
    s = g / np.sqrt(v + np.float32(EPS))
    if conv + "_bias" in w:                 # legacy conv bias folds into the BN shift
        return (k * s).astype(np.float32), (b + (w[conv + "_bias"].astype(np.float32) - m) * s).astype(np.float32)
    return (k * s).astype(np.float32), (b - m * s).astype(np.float32)


def forward_bf16_emulated(desc, weights, planes):
    assert not getattr(desc, "resnet_v2", False), "v1 only (v2 nets are checked against forward())"
    w = dict(weights)
    leaky = desc.leaky_relu
    x = bf16_round(np.transpose(planes, (0, 2, 3, 1))).astype(np.float64)
    k, b = _fold(w, "initial_conv", "initial_bn")
    x = _act(_conv_same(x, bf16_round(k)) + b, leaky)
    for i in range(desc.residual_layers):
        t = x
        k0, b0 = _fold(w, "res%d_conv0" % i, "res%d_bn0" % i)
        k1, b1 = _fold(w, "res%d_conv1" % i, "res%d_bn1" % i)
        y = _act(_conv_same(bf16_round(x).astype(np.float64), bf16_round(k0)) + b0, leaky)
        y = _conv_same(bf16_round(y).astype(np.float64), bf16_round(k1)) + b1
        x = _act(t + y, leaky)
    outs = []
    for r in range(desc.role_count):
        k, b = _fold(w, "policy%d_conv" % r, "policy%d_bn" % r)
        h = _act(_conv_same(x, k) + b, leaky)
        logits = _flatten(h, desc.flatten_nchw) @ w["policy%d_dense" % r].astype(np.float64)
        outs.append(_softmax(logits + w["policy%d_bias" % r]).astype(np.float32))
    if getattr(desc, "value_bn", False):
        k, b = _fold(w, "value_conv", "value_bn")
        v = _act(_conv_same(x, k) + b, leaky)
    else:
        v = _conv_same(x, w["value_conv"])
        if "value_conv_bias" in w:
            v = v + w["value_conv_bias"]
        v = _act(v, leaky)
    hid = _act(_flatten(v, desc.flatten_nchw) @ w["value_hidden"].astype(np.float64)
               + w["value_hidden_bias"], leaky)
    val = hid @ w["value_dense"].astype(np.float64) + w["value_bias"]
    outs.append(_value_out(desc, val))
    return outs
