"""Network manager (reference src/ggpzero/nn/manager.py:20-139): transformers per game /
generation description, new random-init networks, save / load of (model desc JSON + weight blob)."""
import json
import os

import numpy as np

from .. import sm as sm_mod
from ..defs import datadesc, templates
from .bases import GdlBasesTransformer
from .desc import NetDesc
from .network import HipModel, NeuralNetwork, desc_from_conf
from .weights import from_blob, random_weights, to_blob


class Manager(object):
    def __init__(self, data_path=None, device=0):
        self.data_path = data_path or os.environ.get("GGPZERO_PATH", ".")
        self.device = device
        self.transformers = {}

    def get_transformer(self, game, generation_descr=None):
        if generation_descr is None:
            generation_descr = templates.default_generation_desc(game)
        assert isinstance(generation_descr, datadesc.GenerationDescription)
        d = generation_descr
        key = (game, d.channel_last, d.multiple_policy_heads, d.num_previous_states, d.draw_head)
        t = self.transformers.get(key)
        if t is None:
            t = GdlBasesTransformer(sm_mod.get_sm(game), generation_descr)
            self.transformers[key] = t
        return t

    def create_new_network(self, game, nn_model_conf=None, generation_descr=None, seed=0):
        if generation_descr is None:
            generation_descr = templates.default_generation_desc(game)
        transformer = self.get_transformer(game, generation_descr)
        if nn_model_conf is None or isinstance(nn_model_conf, str):
            nn_model_conf = templates.nn_model_config_template(game, nn_model_conf or "small", transformer)
        desc = desc_from_conf(nn_model_conf, generation_descr)
        model = HipModel(desc, random_weights(desc, seed), self.device)
        return NeuralNetwork(transformer, model, generation_descr)

    def network_from_desc(self, game, desc, weights, generation_descr):
        transformer = self.get_transformer(game, generation_descr)
        return NeuralNetwork(transformer, HipModel(desc, weights, self.device), generation_descr)

    def network_from_keras(self, game, model_json, layer_weights, generation_descr=None):
        """A reference model file (data/<game>/models/<gen>.json) + its per-layer weights (dict or an
        .npz of '<layer>/<i>' arrays, see nn/keras_model.py) -> NeuralNetwork on the HIP forward.
        Replaces load_network's Keras model_from_json + load_weights (manager.py:129-139)."""
        from . import keras_model
        if isinstance(layer_weights, str):
            layer_weights = keras_model.load_layer_weights_npz(layer_weights)
        desc, weights = keras_model.weights_from_keras(model_json, layer_weights)
        if generation_descr is None:
            generation_descr = templates.default_generation_desc(game, num_previous_states=1,
                                                                 draw_head=desc.num_values == 3)
        return self.network_from_desc(game, desc, weights, generation_descr)

    def _path(self, game, sub, name, ext):
        p = os.path.join(self.data_path, game, sub)
        os.makedirs(p, exist_ok=True)
        return os.path.join(p, name + ext)

    def save_network(self, nn, generation_name=None):
        game = nn.generation_descr.game
        name = generation_name or nn.generation_descr.name
        desc = nn.get_model().desc
        with open(self._path(game, "models", name, ".gz.json"), "w") as f:
            json.dump(desc.__dict__, f)
        np.save(self._path(game, "weights", name, ".npy"), to_blob(nn.get_model().weights))
        with open(self._path(game, "generations", name, ".json"), "w") as f:
            json.dump(nn.generation_descr.__dict__, f)

    def load_network(self, game, generation_name):
        with open(self._path(game, "generations", generation_name, ".json")) as f:
            gen = datadesc.GenerationDescription(**json.load(f))
        with open(self._path(game, "models", generation_name, ".gz.json")) as f:
            desc = NetDesc(**json.load(f))
        blob = np.load(self._path(game, "weights", generation_name, ".npy"), allow_pickle=False)
        return self.network_from_desc(game, desc, from_blob(desc, blob), gen)


_the_manager = None


def get_manager():
    global _the_manager
    if _the_manager is None:
        _the_manager = Manager()
    return _the_manager
