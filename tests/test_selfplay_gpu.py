"""GPU self-play: the drop-in poll path (cppinterface.Supervisor + NeuralNetwork on the fused HIP
forward) replayed through the oracle must give bit-identical planes and samples; the native
multi-threaded runner must run cleanly and be deterministic per game."""
import numpy as np
import pytest

from galvanise_zero_amd import cppinterface
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.network import HipModel, NeuralNetwork
from puct_harness import Setup, run_oracle_supervisor, sample_key

pytestmark = pytest.mark.gpu


class RecordingModel(object):
    def __init__(self, model):
        self.model = model
        self.planes, self.outs = [], []

    def predict_on_batch(self, X):
        out = self.model.predict_on_batch(X)
        self.planes.append(np.array(X, copy=True).reshape(-1))
        self.outs.append([np.array(o, copy=True) for o in out])
        return out


def _conf(evals=16):
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    conf.puct_config.backup_finalised = True
    conf.run_to_end_puct_config.backup_finalised = True
    return conf


def test_dropin_supervisor_gpu_matches_oracle(hip_device):
    setup = Setup("breakthroughSmall")
    model = RecordingModel(HipModel(setup.desc, setup.weights, hip_device))
    nn = NeuralNetwork(setup.transformer, model, None)
    sup = cppinterface.Supervisor(setup.sm, nn, batch_size=4, seed=7, per_pool_unique_states=True,
                                  identifier="t")
    sup.c_supervisor.set_sample_interval(1)
    conf = _conf()
    sup.start_self_play(conf, 0)
    polls = 1200
    for _ in range(polls):
        assert sup.poll() == sup.POLL_AGAIN
    samples = [s.__dict__ for s in sup.fetch_samples()]

    # oracle replay with the GPU's outputs
    outs = iter(model.outs)

    setup.nn = lambda planes: next(outs)
    olog, osamples, _ = run_oracle_supervisor(setup, conf, 4, polls, seed=7, native_log=model.planes)
    assert len(olog) == polls
    assert [sample_key(setup, s, True) for s in samples] == [sample_key(setup, s, False) for s in osamples]
    assert len(samples) > 10


def test_native_runner_runs(hip_device):
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.weights import to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    setup = Setup("breakthroughSmall")
    net = HipNet(setup.desc, hip_device)
    net.set_weights(to_blob(setup.weights))
    r = SelfPlayRunner(net, setup.sm, setup.transformer, _conf(), device=hip_device, num_threads=2,
                       pools_per_thread=2, batch_size=32, seed=3, keep_samples=True)
    r.start()
    r.wait_rows(4000 * 32, timeout_s=240)
    r.stop()
    st = r.stats()
    samples = r.fetch_samples()
    r.close()
    assert st["rows"] >= 4000 * 32 and st["batches"] > 0
    assert st["kernel_launches"] == st["batches"] and st["kernel_ms"] > 0
    assert st["batches"] <= st["segments"] <= 4 * st["batches"]     # 4 pools, merged launches
    assert st["games_completed"] > 0
    assert len(samples) == st["samples"] > 0
    s0 = samples[0]
    for key in ("state", "prev_states", "policies", "final_score", "depth", "game_length", "match_identifier",
                "has_resigned", "resign_false_positive", "starting_sample_depth", "resultant_puct_score",
                "resultant_puct_visits"):
        assert key in s0, key
