"""Network description + canonical weight-blob layout of the residual policy/value CNN.

Restates the topologies built by ``get_network_model`` (reference ``src/ggpzero/nn/model.py:154-296``).
v1 (``resnet_v2=False``, AlphaGo-Zero style; every BASELINE config):

* initial ``conv2d_block(F, k, use_bias=False) -> BN -> act``            (model.py:205-208, 25-44)
* ``residual_layers`` x ``residual_block_v1``: conv-BN-act-conv-BN-add-act (model.py:47-75)

v2 (``resnet_v2=True``, pre-activation; the reference's ``features=True`` templates and its non-legacy
model files, e.g. data/breakthroughSmall/models/b1_58.json):

* initial ``conv2d_block(F, 1)`` -> BN -> act (model.py:176-179); older model files have a bare 1x1
  conv there (``initial_bn=False``: no BN, no activation)
* ``residual_layers`` x ``residual_block_v2(num_convs=2)``: BN-act-conv-BN-act-conv, optional
  squeeze-excite gate (GlobalAveragePooling -> Dense(S, relu, no bias) -> Dense(F, sigmoid, no bias)
  -> multiply), add -- no activation after the add (model.py:78-151); dropout is inference-identity
* the heads read the last add directly (no final BN / activation)

Heads (both):

* per role: ``conv2d_block(2, 1)`` -> BN -> act -> Flatten -> Dense(P_r, softmax)  (model.py:223-241)
* value:  ``conv2d_block(1, 1, do_bn=False)`` -> act -> Flatten -> Dense(hidden, act)
  -> Dense(V, softmax)                                                     (model.py:273-291);
  with ``global_pooling_value`` the value 1x1 conv has BN and the flat features are
  [GlobalAveragePooling(trunk) (F), conv (HW)] concatenated in that order (model.py:262-271);
  with ``concat_all_layers`` (v2 only) every trunk layer -- the initial conv block's output and each
  residual block's add -- gets its own ``conv2d_block(1, 1)`` (conv + BN + act), and the flat
  features are those B + 1 maps of HW values concatenated in layer order (model.py:251-260)

BatchNormalization is inference-mode with epsilon 1e-3 (Keras default; every
``data/*/models/*.json`` records ``epsilon: 0.001``).

The canonical blob is the concatenation, in the order of :func:`weight_spec`, of float32 tensors in
Keras storage layout (conv kernels HWIO ``[kh][kw][cin][cout]``, dense ``[in][out]``).  This is the
order a Keras ``model.get_weights()`` of the reference model produces once the BN tensors are
grouped as (gamma, beta, moving_mean, moving_variance).  The C-ABI ``gz_net_set_weights``
(``include/gzero_nn.h``) consumes exactly this blob.
"""

from dataclasses import dataclass, field
from typing import List, Tuple

BN_EPSILON = 1e-3
LEAKY_ALPHA = 0.03          # klayers.LeakyReLU(alpha=0.03), model.py:13


@dataclass
class NetDesc:
    """Mirror of the fields of ``confs.NNModelConfig`` (confs.py:127-151) the forward needs."""
    input_channels: int
    input_columns: int          # H = len(y_cords)  (bases.py:115-121)
    input_rows: int             # W = len(x_cords)
    cnn_filter_size: int
    residual_layers: int
    policy_dist_count: List[int]
    value_hidden_size: int = 256
    num_values: int = 2         # 3 with a draw head (model.py:246-249)
    cnn_kernel_size: int = 3
    leaky_relu: bool = False
    # Keras >= 2.1.6 Flatten under channels_first permutes to (H, W, C) before flattening; the
    # legacy (keras 2.1.3) model files flatten in (C, H, W) order.  See SURVEY appendix A.
    flatten_nchw: bool = False
    # Legacy v1 model files (keras 2.1.3-2.1.5, e.g. data/breakthrough/models/x6_102.json): every
    # Conv2D carries a bias, the value head's 1x1 conv is followed by BatchNormalization, and the
    # value Dense uses sigmoid.  Off for the current model.py (use_bias=False, model.py:25-44,
    # value conv do_bn=False :275-279, softmax :287-291).
    conv_bias: bool = False
    value_bn: bool = False
    value_sigmoid: bool = False
    # v2 (pre-activation) trunk, model.py:78-151, 171-198
    resnet_v2: bool = False
    initial_bn: bool = True          # v2 initial 1x1 conv followed by BN + act (False: bare conv)
    se_units: int = 0                # squeeze-excite compress units (0: no SE; model.py: F // 3)
    global_pooling_value: bool = False
    # initial conv kernel: 0 = model.py's (1 for v2, cnn_kernel_size for v1); some v2 model files
    # (e.g. data/hexLG13/models/b4_305.json) have a 3x3 initial conv + BN + act
    initial_kernel_size: int = 0
    # value head over every trunk layer (model.py:251-260; v2 only, e.g. data/hex19/models/h2_477.json)
    concat_all_layers: bool = False

    @property
    def initial_kernel(self):
        if self.initial_kernel_size:
            return self.initial_kernel_size
        return 1 if self.resnet_v2 else self.cnn_kernel_size

    @property
    def value_features(self):
        """Inputs of the value hidden Dense: [GAP (F)] + the value conv's HW, or (B + 1) HW with
        concat_all_layers."""
        if self.concat_all_layers:
            return (self.residual_layers + 1) * self.hw
        return (self.cnn_filter_size if self.global_pooling_value else 0) + self.hw

    @property
    def role_count(self):
        return len(self.policy_dist_count)

    @property
    def hw(self):
        return self.input_columns * self.input_rows

    def flops_per_eval(self):
        """Algorithmic FLOPs (2/MAC) of one leaf evaluation, BN/act/softmax excluded."""
        f = self.flops_trunk()
        for p in self.policy_dist_count:
            f += 2 * (2 * self.hw) * p
        f += 2 * self.value_features * self.value_hidden_size + 2 * self.value_hidden_size * self.num_values
        return f

    def flops_trunk(self):
        """FLOPs of the trunk kernel per evaluation: every conv incl. the heads' 1x1 convs, and the
        squeeze-excite dense layers."""
        F, C, HW, k, k0 = self.cnn_filter_size, self.input_channels, self.hw, self.cnn_kernel_size, self.initial_kernel
        f = 2 * HW * C * F * k0 * k0 + self.residual_layers * 2 * (2 * HW * F * F * k * k)
        f += self.residual_layers * 2 * (2 * F * self.se_units)
        value_convs = self.residual_layers + 1 if self.concat_all_layers else 1
        return f + (2 * self.role_count + value_convs) * 2 * HW * F

    def flops_heads(self):
        """FLOPs of the heads kernel per evaluation: the dense layers."""
        return self.flops_per_eval() - self.flops_trunk()


def weight_spec(d: NetDesc) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) list of the canonical float32 weight blob."""
    F, C, k = d.cnn_filter_size, d.input_channels, d.cnn_kernel_size
    spec = []

    def bn(prefix, n):
        spec.extend([(prefix + "_gamma", (n,)), (prefix + "_beta", (n,)),
                     (prefix + "_mean", (n,)), (prefix + "_var", (n,))])

    def conv(name, shape):
        spec.append((name, shape))
        if d.conv_bias:                     # Keras Conv2D weights: [kernel, bias]
            spec.append((name + "_bias", (shape[3],)))

    k0 = d.initial_kernel
    conv("initial_conv", (k0, k0, C, F))
    if d.initial_bn or not d.resnet_v2:
        bn("initial_bn", F)
    for i in range(d.residual_layers):
        if d.resnet_v2:                      # BN-act-conv-BN-act-conv [SE] add   (model.py:128-149)
            bn("res%d_bn1" % i, F)
            conv("res%d_conv1" % i, (k, k, F, F))
            bn("res%d_bn2" % i, F)
            conv("res%d_conv2" % i, (k, k, F, F))
            if d.se_units:
                spec.append(("res%d_se_compress" % i, (F, d.se_units)))
                spec.append(("res%d_se_gating" % i, (d.se_units, F)))
        else:
            conv("res%d_conv0" % i, (k, k, F, F))
            bn("res%d_bn0" % i, F)
            conv("res%d_conv1" % i, (k, k, F, F))
            bn("res%d_bn1" % i, F)
    for r, p in enumerate(d.policy_dist_count):
        conv("policy%d_conv" % r, (1, 1, F, 2))
        bn("policy%d_bn" % r, 2)
        spec.append(("policy%d_dense" % r, (2 * d.hw, p)))
        spec.append(("policy%d_bias" % r, (p,)))
    if d.concat_all_layers:                  # one conv2d_block(1, 1) per trunk layer (model.py:251-260)
        for j in range(d.residual_layers + 1):
            conv("value%d_conv" % j, (1, 1, F, 1))
            bn("value%d_bn" % j, 1)
    else:
        conv("value_conv", (1, 1, F, 1))
        if d.value_bn:
            bn("value_bn", 1)
    spec.append(("value_hidden", (d.value_features, d.value_hidden_size)))
    spec.append(("value_hidden_bias", (d.value_hidden_size,)))
    spec.append(("value_dense", (d.value_hidden_size, d.num_values)))
    spec.append(("value_bias", (d.num_values,)))
    return spec


def blob_size(d: NetDesc) -> int:
    n = 0
    for _, shape in weight_spec(d):
        c = 1
        for s in shape:
            c *= s
        n += c
    return n


# BASELINE.json configs.  C, P_r from the reference model JSONs with
# num_previous_states=1; net sizes from BASELINE.json.
BASELINE_CONFIGS = {
    1: dict(game="breakthroughSmall", desc=NetDesc(5, 6, 6, 64, 2, [81, 81]), evals=100),
    2: dict(game="breakthrough", desc=NetDesc(5, 8, 8, 128, 6, [155, 155]), evals=800, batch=256),
    3: dict(game="reversi", desc=NetDesc(5, 8, 8, 128, 10, [65, 65], num_values=3), evals=800),
    4: dict(game="hexLG13", desc=NetDesc(5, 13, 13, 256, 12, [170, 171]), evals=1600),
    5: dict(game="amazons_10x10", desc=NetDesc(12, 10, 10, 256, 20, [3041, 3041]), evals=1600),
}
