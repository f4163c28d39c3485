"""Drives the native engine (C-ABI) and the oracle (oracle/puct_ref.py) through the reference's
poll protocol with the same network outputs, recording every batch of planes."""
import numpy as np

from galvanise_zero_amd import cppinterface
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.bases import GdlBasesTransformer
from galvanise_zero_amd.nn.desc import NetDesc
from galvanise_zero_amd.nn.weights import random_weights
from galvanise_zero_amd.sm import get_sm
from oracle import games_ref, nn_ref, planes_ref
from oracle import puct_ref as P


class Setup(object):
    def __init__(self, game, num_prev_states=1, wseed=5, bias_std=0.3, draw_head=False):
        self.game = game
        self.sm = get_sm(game)
        gen = templates.default_generation_desc(game, num_previous_states=num_prev_states, draw_head=draw_head)
        self.transformer = GdlBasesTransformer(self.sm, gen)
        t = self.transformer
        self.desc = NetDesc(t.num_channels, t.num_cols, t.num_rows, 16 * 4, 1, list(t.policy_dist_count),
                            value_hidden_size=32, num_values=t.num_rewards)
        self.weights = random_weights(self.desc, wseed, bias_std=bias_std)
        self.ref_sm = games_ref.make(game)
        self.ref_planes = planes_ref.Planes(game, [self.sm.base_name(i) for i in range(self.sm.num_bases)],
                                            num_prev_states)
        self.num_prev_states = num_prev_states

    def nn(self, planes_flat):
        t = self.transformer
        n = planes_flat.size // (t.num_channels * t.channel_size)
        x = np.asarray(planes_flat, dtype=np.float32).reshape(n, t.num_channels, t.num_cols, t.num_rows)
        return nn_ref.forward(self.desc, self.weights, x)

    def empty_arrays(self):
        return [np.zeros(0, dtype=np.float32) for _ in range(self.sm.role_count + 1)]


def run_native_supervisor(setup, conf, batch, polls, seed, workers=0):
    ct = cppinterface.create_c_transformer(setup.transformer)
    sup = cppinterface._CSupervisor(setup.sm, ct, batch, "t", seed=seed, per_pool_unique_states=True)
    sup.set_sample_interval(1)
    sup.start_self_play(workers, conf)
    arrays = setup.empty_arrays()
    log = []
    for _ in range(polls):
        buf = sup.poll(len(arrays[0]), arrays)
        if buf is None:
            break
        buf = np.array(buf, copy=True)
        log.append(buf)
        arrays = setup.nn(buf)
    samples = sup.fetch_samples() or []
    return log, samples, sup.stats(), (sup, ct)


def run_oracle_supervisor(setup, conf, batch, polls, seed, native_log=None):
    t = setup.transformer
    man = P.Manager(setup.ref_sm, setup.ref_planes, batch,
                    P.UniqueStates(setup.ref_planes.hash_mask(), 1000), "t_inline", seed, 0,
                    list(t.policy_dist_count), t.num_rewards, setup.num_prev_states)
    man.start(conf)
    pred = (0, [np.zeros(0, np.float32)] * setup.sm.role_count, np.zeros(0, np.float32))
    log = []
    for i in range(polls):
        buf = man.poll(*pred)
        if buf is None:
            break
        log.append(buf)
        if native_log is not None:
            assert i < len(native_log) and np.array_equal(buf, native_log[i]), "planes diverged at poll %d" % i
        outs = setup.nn(buf)
        pred = (outs[0].shape[0], outs[:-1], outs[-1])
    return log, man.samples, man


def sample_key(setup, s, native):
    """Normalise a sample (native JSON dict or oracle dict) for exact comparison."""
    if native:
        state = games_ref.words_to_state(setup.sm.from_bits(s["state"]))
        prev = [games_ref.words_to_state(setup.sm.from_bits(p)) for p in s["prev_states"]]
        pols = [[(int(a), float(np.float32(p))) for a, p in pol] for pol in s["policies"]]
    else:
        state, prev = s["state"], s["prev_states"]
        pols = [[(int(a), float(np.float32(p))) for a, p in pol] for pol in s["policies"]]
    return (state, tuple(prev), tuple(tuple(p) for p in pols),
            tuple(float(np.float32(x)) for x in s["final_score"]), s["depth"], s["game_length"],
            s["match_identifier"], bool(s["has_resigned"]), bool(s["resign_false_positive"]),
            s["starting_sample_depth"], tuple(float(np.float32(x)) for x in s["resultant_puct_score"]),
            s["resultant_puct_visits"])
