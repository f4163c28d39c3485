"""GPU self-play: the drop-in poll path (cppinterface.Supervisor + NeuralNetwork on the fused HIP
forward) replayed through the oracle must give bit-identical planes and samples; the native
multi-threaded runner must run cleanly and be deterministic per game."""
import json

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


@pytest.mark.parametrize("game", ["breakthroughSmall", "reversi", "breakthrough_cfg2"])
def test_dropin_supervisor_gpu_matches_oracle(game, hip_device):
    """breakthrough_cfg2: BASELINE configs[1]'s game on its 6-block x 128-filter net."""
    cfg2 = game == "breakthrough_cfg2"
    game = "breakthrough" if cfg2 else game
    setup = Setup(game, draw_head=(game == "reversi"))
    if cfg2:
        from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
        from galvanise_zero_amd.nn.weights import random_weights
        setup.desc = BASELINE_CONFIGS[2]["desc"]
        setup.weights = random_weights(setup.desc, 7921)
    model = RecordingModel(HipModel(setup.desc, setup.weights, hip_device))
    nn = NeuralNetwork(setup.transformer, model, None)
    sup = cppinterface.Supervisor(setup.sm, nn, batch_size=4, seed=7, per_pool_unique_states=True,
                                  identifier="t")
    sup.c_supervisor.set_sample_interval(1)
    conf = _conf()
    sup.start_self_play(conf, 0)
    polls = {"breakthroughSmall": 1200, "reversi": 2500, "breakthrough": 2000}[game]
    for _ in range(polls):
        assert sup.poll() == sup.POLL_AGAIN
    samples = [s.__dict__ for s in sup.fetch_samples()]

    # oracle replay with the GPU's outputs
    outs = iter(model.outs)

    setup.nn = lambda planes: next(outs)
    olog, osamples, _ = run_oracle_supervisor(setup, conf, 4, polls, seed=7, native_log=model.planes)
    assert len(olog) == polls
    assert [sample_key(setup, s, True) for s in samples] == [sample_key(setup, s, False) for s in osamples]
    if game != "reversi":
        assert len(samples) > 5


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


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_native_runner_other_games(cfg, hip_device):
    """reversi (draw head), hexLG13 (asymmetric policy heads), amazons_10x10 (12 planes, 3041
    moves) through the native runner on the F=128 / F=256 kernels of their BASELINE geometry
    (2 residual blocks instead of 10-20 to keep the test short); runs twice with the same seed
    and must produce the same samples."""
    from dataclasses import replace
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.defs import templates as T
    from galvanise_zero_amd.nn.bases import GdlBasesTransformer
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    from galvanise_zero_amd.sm import get_sm
    c = BASELINE_CONFIGS[cfg]
    desc = replace(c["desc"], residual_layers=2)
    sm = get_sm(c["game"])
    t = GdlBasesTransformer(sm, T.default_generation_desc(c["game"], num_previous_states=1,
                                                          draw_head=desc.num_values == 3))
    assert (t.num_channels, t.num_cols, t.num_rows, list(t.policy_dist_count), t.num_rewards) == \
        (desc.input_channels, desc.input_columns, desc.input_rows, list(desc.policy_dist_count), desc.num_values)
    net = HipNet(desc, hip_device)
    net.set_weights(to_blob(random_weights(desc, 11)))
    conf = _conf(8)
    conf.run_to_end_evals = 4
    runs = []
    nbatch = 1500 if cfg == 3 else 300
    for _ in range(2):
        r = SelfPlayRunner(net, sm, t, conf, device=hip_device, num_threads=1, pools_per_thread=1,
                           batch_size=16, seed=9, keep_samples=True)
        r.start()
        r.wait_rows(16 * nbatch, timeout_s=100)
        r.stop()
        st = r.stats()
        samples = r.fetch_samples()
        r.close()
        assert st["rows"] >= 16 * nbatch and st["kernel_launches"] > 0
        runs.append((st, samples))
    # per-game RNG streams + batch-invariant forward: a sample present in both runs is identical
    k0 = {(x["match_identifier"], x["depth"]): json.dumps(x, sort_keys=True) for x in runs[0][1]}
    k1 = {(x["match_identifier"], x["depth"]): json.dumps(x, sort_keys=True) for x in runs[1][1]}
    common = set(k0) & set(k1)
    assert all(k0[k] == k1[k] for k in common)
    if cfg == 3:
        assert runs[0][0]["games_completed"] > 0 and len(common) > 0
