"""Synthetic (random-init) weights for the v1 residual CNN, in the canonical blob layout.

The reference's trained ``.h5`` weights are absent (``.MISSING_LARGE_BLOBS``), so every measured
network here is random-init with the architecture of the BASELINE config.  Distributions follow
SURVEY 8(d) "Synthetic inputs": conv He-normal, BN gamma~U(0.5,1.5), beta~N(0,0.1),
mean~N(0,0.1), var~U(0.5,1.5), Dense Glorot-uniform.  Biases default to 0 as in Keras' default
initialiser; tests pass ``bias_std>0`` to exercise the bias paths.
"""

import numpy as np

from .desc import NetDesc, weight_spec


def random_weights(desc: NetDesc, seed: int, bias_std: float = 0.0, res_gamma: float = 1.0):
    """Returns an ordered dict-like list [(name, float32 array)] following weight_spec().

    ``res_gamma`` scales the branch each residual block adds to the skip path: the gamma of the v1
    block's second BN, the v2 block's second conv kernel.  At 1.0 the residual stream of a deep random net grows with depth until every softmax
    saturates (outputs 0/1), which hides numerical differences; parity tests of the 10-20 block
    configs use 0.15 so the outputs stay in the interior.
    """
    rng = np.random.default_rng(seed)
    out = []
    for name, shape in weight_spec(desc):
        if len(shape) == 4:  # conv kernels, HWIO
            fan_in = shape[0] * shape[1] * shape[2]
            w = rng.normal(0.0, np.sqrt(2.0 / fan_in), size=shape)
            if desc.resnet_v2 and name.endswith("_conv2"):
                w = w * res_gamma
        elif name.endswith("_gamma"):
            w = rng.uniform(0.5, 1.5, size=shape)
            if name.endswith("_bn1_gamma"):
                w = w * res_gamma
        elif name.endswith("_beta") or name.endswith("_mean"):
            w = rng.normal(0.0, 0.1, size=shape)
        elif name.endswith("_var"):
            w = rng.uniform(0.5, 1.5, size=shape)
        elif len(shape) == 2:
            limit = np.sqrt(6.0 / (shape[0] + shape[1]))
            w = rng.uniform(-limit, limit, size=shape)
        else:  # dense biases
            w = rng.normal(0.0, bias_std, size=shape) if bias_std > 0 else np.zeros(shape)
        out.append((name, w.astype(np.float32)))
    return out


def to_blob(weights) -> np.ndarray:
    """Concatenate named weights into the canonical contiguous float32 blob."""
    return np.ascontiguousarray(np.concatenate([w.reshape(-1) for _, w in weights]).astype(np.float32))


def from_blob(desc: NetDesc, blob: np.ndarray):
    out, off = [], 0
    for name, shape in weight_spec(desc):
        n = int(np.prod(shape))
        out.append((name, blob[off:off + n].reshape(shape)))
        off += n
    assert off == blob.size, (off, blob.size)
    return out


def random_planes(desc: NetDesc, n: int, seed: int, control_values=(0.0, 1.0)) -> np.ndarray:
    """Synthetic board-plane batch [n, C, H, W] float32.

    Each cell of each state (current + previous) is empty w.p. 0.5 else one of the K piece
    channels (one-hot across that state's piece planes); the control planes are flood-filled with
    one value from the game's control values.
    """
    rng = np.random.default_rng(seed)
    C, H, W = desc.input_channels, desc.input_columns, desc.input_rows
    x = np.zeros((n, C, H, W), dtype=np.float32)
    # breakthrough-like layout: 2 piece channels per state, (C-1)/2 states, 1 control channel
    n_ctrl = 1 if C % 2 == 1 else 4
    per_state = 2 if n_ctrl == 1 else 4
    n_states = (C - n_ctrl) // per_state
    for s in range(n_states):
        occ = rng.random((n, H, W)) < 0.5
        which = rng.integers(0, per_state, size=(n, H, W))
        for k in range(per_state):
            x[:, s * per_state + k] = (occ & (which == k)).astype(np.float32)
    if n_ctrl == 1:
        v = rng.choice(np.array(control_values, dtype=np.float32), size=n)
        x[:, C - 1] = v[:, None, None]
    else:
        t = rng.integers(0, n_ctrl, size=n)
        for i in range(n):
            x[i, C - n_ctrl + t[i]] = 1.0
    return x
