"""ORACLE (test infrastructure only) -- float32 torch-CPU restatement of the reference policy/value
CNN forward, for bench.py's cpu_baseline leg (the reference's CPU self-play design with a CPU
network: SURVEY 8d "CPU path timed beside it").

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (galvanise_zero_amd) never does.

Same layer semantics as oracle/nn_ref.forward (reference src/ggpzero/nn/model.py:25-75, 154-296 as
executed by Keras predict_on_batch, cppinterface.py:119): conv 'same' without bias (legacy files:
with bias), inference BatchNormalization eps 1e-3, ReLU / LeakyReLU(0.03), residual v1 blocks,
policy heads conv1x1(2)+BN+act -> Flatten -> Dense softmax, value head conv1x1(1)(+BN legacy)+act
-> Flatten -> Dense+act -> Dense softmax (legacy: sigmoid).  float32 throughout, like TF's CPU
kernels; NCHW with torch's own conv algorithms.
"""
import numpy as np
import torch
import torch.nn.functional as tF

EPS = 1e-3


class TorchCPUNet(object):
    """predict_on_batch(X[N,C,H,W] float32) -> [policy_0, ..., policy_{R-1}, value] float32."""

    def __init__(self, desc, weights):
        self.desc = desc
        w = {k: torch.tensor(np.asarray(v), dtype=torch.float32) for k, v in weights}
        self.w = w
        self.act = (lambda t: tF.leaky_relu(t, 0.03)) if desc.leaky_relu else tF.relu
        # Keras HWIO kernels -> torch OIHW, once
        self.k = {name: t.permute(3, 2, 0, 1).contiguous() for name, t in w.items() if t.dim() == 4}

    def _conv(self, x, name):
        k = self.k[name]
        b = self.w.get(name + "_bias") if getattr(self.desc, "conv_bias", False) else None
        return tF.conv2d(x, k, bias=b, padding=k.shape[-1] // 2)

    def _bn(self, x, p):
        w = self.w
        return tF.batch_norm(x, w[p + "_mean"], w[p + "_var"], w[p + "_gamma"], w[p + "_beta"],
                             training=False, eps=EPS)

    def _flat(self, t):
        if not self.desc.flatten_nchw:
            t = t.permute(0, 2, 3, 1)
        return t.reshape(t.shape[0], -1)

    def predict_on_batch(self, X):
        d, w, act = self.desc, self.w, self.act
        with torch.inference_mode():
            x = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
            x = act(self._bn(self._conv(x, "initial_conv"), "initial_bn"))
            for i in range(d.residual_layers):
                y = act(self._bn(self._conv(x, "res%d_conv0" % i), "res%d_bn0" % i))
                y = self._bn(self._conv(y, "res%d_conv1" % i), "res%d_bn1" % i)
                x = act(x + y)
            outs = []
            for r in range(d.role_count):
                h = act(self._bn(self._conv(x, "policy%d_conv" % r), "policy%d_bn" % r))
                z = self._flat(h) @ w["policy%d_dense" % r] + w["policy%d_bias" % r]
                outs.append(torch.softmax(z, 1).numpy())
            v = self._conv(x, "value_conv")
            if getattr(d, "value_bn", False):
                v = self._bn(v, "value_bn")
            v = act(v)
            hid = act(self._flat(v) @ w["value_hidden"] + w["value_hidden_bias"])
            z = hid @ w["value_dense"] + w["value_bias"]
            outs.append((torch.sigmoid(z) if getattr(d, "value_sigmoid", False) else torch.softmax(z, 1)).numpy())
        return outs
