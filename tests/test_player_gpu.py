"""Match play on the MI355X forward (reference player/puctplayer.py:13-108,
cppinterface.py:156-182, evaluator.cpp:1058-1069): PlayPoller at the reference's match setting,
in-tree batch_size 32 with more than 100 evaluations per move (so the 31 virtual-loss playout
workers spawn), on the BASELINE configs[1] net in both arithmetic modes.  The oracle player
(oracle/puct_ref.Player) is driven in lockstep with the same network outputs; planes at every poll,
the chosen move and every root child's visits and policy must be identical."""
import numpy as np
import pytest

from galvanise_zero_amd.defs import confs, templates
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
from galvanise_zero_amd.nn.network import HipModel, NeuralNetwork
from galvanise_zero_amd.nn.weights import random_weights
from galvanise_zero_amd.player.puctplayer import PUCTPlayer, play_match
from puct_harness import Setup
from test_puct_parity import _player_run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["bf16x3", "bf16"])
def test_player_batch32_gpu_bit_exact(precision, hip_device):
    setup = Setup("breakthrough")
    setup.desc = BASELINE_CONFIGS[2]["desc"]
    setup.weights = random_weights(setup.desc, 7921)
    model = HipModel(setup.desc, setup.weights, hip_device, precision)
    setup.nn = lambda planes: model.predict_on_batch(
        np.asarray(planes, np.float32).reshape(-1, setup.desc.input_channels, setup.desc.input_columns,
                                               setup.desc.input_rows))
    conf = templates.base_puct_config(batch_size=32, choose="choose_temperature", dirichlet_noise_pct=0.25,
                                      think_time=-1, converged_visits=1)
    visits = _player_run(setup, conf, 160, 3, seed=17)
    assert sum(t for _, t, _ in visits[0]) > 100


def test_puctplayer_match_on_gpu(hip_device):
    """A full breakthroughSmall match between two PUCTPlayers on HipModel (batch 32 and 1)."""
    setup = Setup("breakthroughSmall")
    desc = BASELINE_CONFIGS[1]["desc"]
    w = random_weights(desc, 5)

    def player(batch, playouts, seed):
        ev = templates.base_puct_config(batch_size=batch, choose="choose_temperature", dirichlet_noise_pct=0.25,
                                        think_time=-1, converged_visits=1)
        conf = confs.PUCTPlayerConfig(name="gpu%d" % batch, playouts_per_iteration=playouts, generation="test",
                                      evaluator_config=ev)
        nn = NeuralNetwork(setup.transformer, HipModel(desc, w, hip_device, "bf16x3"), None)
        return PUCTPlayer(conf, nn=nn, seed=seed)

    goals, moves = play_match("breakthroughSmall", [player(32, 200, 3), player(1, 64, 4)])
    assert sorted(goals) == [0, 100] and len(moves) > 5
