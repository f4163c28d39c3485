"""NeuralNetwork wrapper (reference src/ggpzero/nn/network.py:10-165) whose model runs on the
MI355X fused HIP forward.  ``get_model().predict_on_batch(X)`` keeps the Keras contract used by
the poll loop (cppinterface.py:119): X float32 [N, C, H, W] -> [policy_0 .. policy_{R-1}, value]."""
import numpy as np

from .._native import HipNet
from .desc import NetDesc
from .weights import to_blob


def desc_from_conf(nn_model_conf, generation_descr=None):
    """NNModelConfig (+ GenerationDescription.draw_head) -> NetDesc, as get_network_model builds it
    (model.py:154-296): v1, or v2 with squeeze-excite (ratio 3, :190-197) and the global-pooling
    value head (whose 1x1 conv has BN, :265-268)."""
    c = nn_model_conf
    if c.concat_all_layers and (not c.resnet_v2 or c.global_pooling_value):
        raise ValueError("concat_all_layers needs resnet_v2 and no global_pooling_value (model.py:170-252)")
    if c.squeeze_excite_layers and not c.resnet_v2:
        raise ValueError("squeeze_excite_layers needs resnet_v2 (model.py:202)")
    se = c.cnn_filter_size // 3 if (c.resnet_v2 and c.squeeze_excite_layers) else 0
    if se:
        assert se > 8, "model.py:111: filter_size // ratio > 8"
    draw = bool(generation_descr is not None and generation_descr.draw_head)
    return NetDesc(input_channels=c.input_channels, input_columns=c.input_columns, input_rows=c.input_rows,
                   cnn_filter_size=c.cnn_filter_size, residual_layers=c.residual_layers,
                   policy_dist_count=list(c.policy_dist_count), value_hidden_size=c.value_hidden_size,
                   num_values=3 if draw else 2, cnn_kernel_size=c.cnn_kernel_size, leaky_relu=c.leaky_relu,
                   resnet_v2=bool(c.resnet_v2), se_units=se, global_pooling_value=bool(c.global_pooling_value),
                   value_bn=bool(c.global_pooling_value), concat_all_layers=bool(c.concat_all_layers))


class HipModel(object):
    """Model object with the Keras inference surface the hot path uses."""

    def __init__(self, desc, weights, device=0, precision="bf16"):
        self.desc = desc
        self.weights = weights
        self.net = HipNet(desc, device, precision)
        self.net.set_weights(to_blob(weights))

    def predict_on_batch(self, X):
        X = np.asarray(X, dtype=np.float32)
        d = self.desc
        assert X.shape[1:] == (d.input_channels, d.input_columns, d.input_rows), X.shape
        return self.net.forward(X)

    def predict(self, X, batch_size=None):
        return self.predict_on_batch(X)

    def set_weights(self, weights):
        self.weights = weights
        self.net.set_weights(to_blob(weights))

    def last_kernel_ms(self):
        return self.net.last_kernel_ms()


class HeadResult(object):
    def __init__(self, transformer, policies, values):
        assert len(transformer.policy_dist_count) == len(policies)
        self.policies = policies
        self.scores = values


class NeuralNetwork(object):
    def __init__(self, gdl_bases_transformer, model, generation_descr):
        self.gdl_bases_transformer = gdl_bases_transformer
        self.model = model
        self.generation_descr = generation_descr

    def get_model(self):
        return self.model

    def predict_n(self, states, prev_states=None):
        to_channels = self.gdl_bases_transformer.state_to_channels
        if prev_states:
            X = np.array([to_channels(s, p) for s, p in zip(states, prev_states)])
        else:
            X = np.array([to_channels(s) for s in states])
        Y = self.model.predict_on_batch(X)
        return [HeadResult(self.gdl_bases_transformer, [Y[k][i] for k in range(len(Y) - 1)], Y[-1][i])
                for i in range(len(states))]

    def predict_1(self, state, prev_states=None):
        return self.predict_n([state], [prev_states] if prev_states else None)[0]
