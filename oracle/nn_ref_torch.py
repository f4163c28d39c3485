"""ORACLE (test infrastructure only) -- oracle/nn_ref.forward restated in float64 torch, so the
float64 reference forward runs on any torch device (the GPU box measures the split kernel's error
distribution at the bench's launch sizes with it: tools/split_error_dist.py).

Only tests/, tools/ measurement scripts, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product path (galvanise_zero_amd) never does.

Same layer semantics, expression by expression, as nn_ref.forward (reference
src/ggpzero/nn/model.py:25-75, 78-151, 154-296): NHWC float64, 'same' convs as shifted matmuls,
inference BatchNormalization eps 1e-3, v1 / v2 trunks, squeeze-excite, the global-pooling and
concat-all-layers value heads.  Pinned against nn_ref.forward by tests/test_nn_oracle.py (CPU,
float64: agreement to ~1e-12).
"""
import numpy as np
import torch

EPS = 1e-3
LEAKY = 0.03


def forward(desc, weights, planes, logits=False, device="cpu"):
    """planes float32 [N, C, H, W] -> [policy_0, ..., policy_{R-1}, value] as numpy (float32, or
    float64 logits with logits=True), like nn_ref.forward."""
    dev = torch.device(device)
    w = {k: torch.as_tensor(np.asarray(v), dtype=torch.float64, device=dev) for k, v in weights}
    leaky = desc.leaky_relu

    def act(x):
        return torch.where(x > 0, x, LEAKY * x) if leaky else torch.clamp_min(x, 0.0)

    def bn(x, p):
        return w[p + "_gamma"] * (x - w[p + "_mean"]) / torch.sqrt(w[p + "_var"] + EPS) + w[p + "_beta"]

    def conv(x, name):
        k = w[name]
        kh, kw = k.shape[0], k.shape[1]
        ph, pw = kh // 2, kw // 2
        N, H, W, _ = x.shape
        xp = torch.nn.functional.pad(x, (0, 0, pw, pw, ph, ph))
        out = torch.zeros((N, H, W, k.shape[3]), dtype=torch.float64, device=dev)
        for dy in range(kh):
            for dx in range(kw):
                out += xp[:, dy:dy + H, dx:dx + W, :] @ k[dy, dx]
        if getattr(desc, "conv_bias", False):
            out = out + w[name + "_bias"]
        return out

    def flatten(x):
        if desc.flatten_nchw:
            x = x.permute(0, 3, 1, 2)
        return x.reshape(x.shape[0], -1)

    x = torch.as_tensor(np.asarray(planes, dtype=np.float32), device=dev).to(torch.float64).permute(0, 2, 3, 1)
    v2 = getattr(desc, "resnet_v2", False)
    x = conv(x, "initial_conv")
    if not v2 or desc.initial_bn:
        x = act(bn(x, "initial_bn"))
    layers = [x]
    for i in range(desc.residual_layers):
        t = x
        if v2:
            y = conv(act(bn(x, "res%d_bn1" % i)), "res%d_conv1" % i)
            y = conv(act(bn(y, "res%d_bn2" % i)), "res%d_conv2" % i)
            if desc.se_units:
                m = y.mean(dim=(1, 2))
                h = torch.clamp_min(m @ w["res%d_se_compress" % i], 0.0)
                y = y * torch.sigmoid(h @ w["res%d_se_gating" % i])[:, None, None, :]
            x = t + y
        else:
            y = act(bn(conv(x, "res%d_conv0" % i), "res%d_bn0" % i))
            y = bn(conv(y, "res%d_conv1" % i), "res%d_bn1" % i)
            x = act(t + y)
        layers.append(x)
    outs = []
    for r in range(desc.role_count):
        h = act(bn(conv(x, "policy%d_conv" % r), "policy%d_bn" % r))
        z = flatten(h) @ w["policy%d_dense" % r] + w["policy%d_bias" % r]
        outs.append(z if logits else torch.softmax(z, 1))
    if getattr(desc, "concat_all_layers", False):
        flat = torch.cat([flatten(act(bn(conv(l, "value%d_conv" % j), "value%d_bn" % j)))
                          for j, l in enumerate(layers)], dim=1)
    else:
        v = conv(x, "value_conv")
        if getattr(desc, "value_bn", False):
            v = bn(v, "value_bn")
        flat = flatten(act(v))
        if getattr(desc, "global_pooling_value", False):
            flat = torch.cat([x.mean(dim=(1, 2)), flat], dim=1)
    hid = act(flat @ w["value_hidden"] + w["value_hidden_bias"])
    z = hid @ w["value_dense"] + w["value_bias"]
    if logits:
        outs.append(z)
    else:
        outs.append(torch.sigmoid(z) if getattr(desc, "value_sigmoid", False) else torch.softmax(z, 1))
    res = [o.cpu().numpy() for o in outs]
    return res if logits else [o.astype(np.float32) for o in res]
