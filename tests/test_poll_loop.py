"""The reference's own self-play interface test, restated (src/test/cpp/test_interface.py:100-181):
supervisor construction at several batch sizes for every game, and `do_test` - self-play through
`poll_loop` with a callback until N samples arrive, inline (batch 1) and with worker threads, then
`reset_stats` and a second `poll_loop` on the same supervisor (resumable, :166-170).  The network
is the oracle's CPU forward on a small net (the reference test needs a GPU and TF)."""
import pytest

from galvanise_zero_amd import cppinterface
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.network import NeuralNetwork
from puct_harness import Setup


class _OracleModel(object):
    def __init__(self, setup):
        self.setup = setup

    def predict_on_batch(self, X):
        return self.setup.nn(X.reshape(-1))


def _supervisor(game, batch_size, workers=None):
    setup = Setup(game, draw_head=(game == "reversi"))
    nn = NeuralNetwork(setup.transformer, _OracleModel(setup), None)
    return cppinterface.Supervisor(setup.sm, nn, batch_size=batch_size, workers=workers, seed=3,
                                   per_pool_unique_states=True), setup


@pytest.mark.parametrize("game", ["breakthroughSmall", "breakthrough", "reversi", "hexLG13", "amazons_10x10"])
@pytest.mark.parametrize("batch_size", [1, 128, 1024])
def test_inline_supervisor_creation(game, batch_size):
    """test_interface.py:100-120."""
    sup, setup = _supervisor(game, batch_size)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    sup.start_self_play(conf, 0)
    assert sup.poll() == sup.POLL_AGAIN
    t = setup.transformer
    assert sup.poll_last[0].shape[0] <= batch_size


def _do_test(batch_size, get_sample_count, num_workers):
    """test_interface.py:147-170."""
    sup, _ = _supervisor("breakthroughSmall", batch_size)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 12
    conf.run_to_end_evals = 4
    sup.start_self_play(conf, num_workers)
    got = []

    def cb():
        got.extend(sup.fetch_samples())
        return len(got) > get_sample_count

    sup.poll_loop(do_stats=True, cb=cb, cb_every_n=10)
    assert len(got) > get_sample_count
    assert sup.num_predictions_calls > 0 and sup.total_predictions >= sup.num_predictions_calls
    assert sup.acc_time_polling > 0 and sup.acc_time_prediction > 0
    # resumable
    first = list(got)
    del got[:]
    sup.reset_stats()
    assert sup.num_predictions_calls == 0 and sup.total_predictions == 0
    sup.poll_loop(do_stats=True, cb=cb, cb_every_n=10)
    assert len(got) > get_sample_count and sup.num_predictions_calls > 0
    ids = set(s.match_identifier for s in got)
    assert all(s.match_identifier for s in first) and ids


def test_inline_one():
    _do_test(batch_size=1, get_sample_count=10, num_workers=0)


def test_inline_batched():
    _do_test(batch_size=16, get_sample_count=30, num_workers=0)


def test_workers_batched():
    _do_test(batch_size=16, get_sample_count=30, num_workers=2)
