"""PUCTPlayer (reference player/puctplayer.py:13-108) over PlayPoller: a full breakthroughSmall
match between two players on the oracle's CPU forward; finishes with a win, is reproducible at a
fixed seed, and uses in-tree batching (PuctConfig.batch_size > 1, the virtual-loss path)."""
from galvanise_zero_amd.defs import confs, templates
from galvanise_zero_amd.nn.network import NeuralNetwork
from galvanise_zero_amd.player.puctplayer import PUCTPlayer, play_match
from puct_harness import Setup


class _OracleModel(object):
    def __init__(self, setup):
        self.setup = setup

    def predict_on_batch(self, X):
        return self.setup.nn(X.reshape(-1))


def _player(setup, batch, playouts, seed):
    ev = templates.base_puct_config(batch_size=batch, choose="choose_temperature", dirichlet_noise_pct=0.25,
                                    think_time=-1, converged_visits=1)
    conf = confs.PUCTPlayerConfig(name="p%d" % batch, playouts_per_iteration=playouts, generation="test",
                                  evaluator_config=ev)
    return PUCTPlayer(conf, nn=NeuralNetwork(setup.transformer, _OracleModel(setup), None), seed=seed)


def _match(seed):
    setup = Setup("breakthroughSmall")
    players = [_player(setup, 1, 24, seed), _player(setup, 8, 32, seed + 1)]
    goals, moves = play_match("breakthroughSmall", players)
    return goals, moves, players


def test_match_completes_and_is_reproducible():
    goals, moves, players = _match(5)
    assert sorted(goals) == [0, 100]
    assert 5 < len(moves) < 200
    assert all(p.last_node_count > 0 for p in players)
    assert players[0].get_name() == "p1_24_test"
    goals2, moves2, _ = _match(5)
    assert (goals2, moves2) == (goals, moves)
