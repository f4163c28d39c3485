"""Python side of the self-play hot path: the reference's ``ggpzero.util.cppinterface`` API
(src/ggpzero/util/cppinterface.py:33-226) over the MI355X-native engine's C-ABI.

Same names, same argument meaning and the same poll protocol:

    supervisor = Supervisor(sm, nn, batch_size=256)
    supervisor.start_self_play(conf, num_workers)
    supervisor.poll_loop(do_stats=True, cb=...)        # predict <-> poll ping-pong
    supervisor.fetch_samples()

``nn`` is a ``galvanise_zero_amd.nn.network.NeuralNetwork`` whose ``get_model().predict_on_batch``
runs the fused HIP forward (libgz_nn.so).  Native code is mandatory: a missing library raises.
"""
import ctypes
import json
import time

import numpy as np

from . import _native
from .defs import confs, datadesc

_FP = ctypes.POINTER(ctypes.c_float)
_U64P = ctypes.POINTER(ctypes.c_uint64)


def sm_to_ptr(sm):
    """cppinterface.py:12-16: the state-machine handle handed to the C side."""
    return sm.handle


def _as_float_arrays(arrays):
    out = [np.ascontiguousarray(a, dtype=np.float32) for a in arrays]
    ptrs = (_FP * len(out))(*[a.ctypes.data_as(_FP) for a in out])
    return out, ptrs


class CTransformer(object):
    """ggpzero_interface.GdlBasesTransformer (gdltransformer_impl.cpp:186-219)."""

    def __init__(self, channel_size, channels_per_state, num_control_channels, num_prev_states,
                 num_rewards, policy_dist_count):
        self.lib = _native.engine_lib()
        ps = (ctypes.c_int * len(policy_dist_count))(*policy_dist_count)
        self.handle = self.lib.gz_transformer_create(channel_size, channels_per_state, num_control_channels,
                                                     num_prev_states, num_rewards, ps, len(policy_dist_count))
        if not self.handle:
            raise RuntimeError(_native.engine_error())
        self.total_size = None

    def add_board_base(self, base_indx, buf_incr):
        self.lib.gz_transformer_add_board_base(self.handle, base_indx, buf_incr)

    def add_control_base(self, base_indx, channel_id, value):
        self.lib.gz_transformer_add_control_base(self.handle, base_indx, channel_id, value)

    def to_channels(self, state, prev_states=()):
        n = self.lib.gz_transformer_total_size(self.handle)
        out = np.empty(n, dtype=np.float32)
        state = np.ascontiguousarray(state, dtype=np.uint64)
        prev = [np.ascontiguousarray(p, dtype=np.uint64) for p in prev_states]
        parr = (_U64P * max(1, len(prev)))(*[p.ctypes.data_as(_U64P) for p in prev])
        self.lib.gz_transformer_to_channels(self.handle, state.ctypes.data_as(_U64P), parr, len(prev),
                                            out.ctypes.data_as(_FP))
        return out

    def __del__(self):
        try:
            if self.handle:
                self.lib.gz_transformer_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def create_c_transformer(transformer):
    """cppinterface.py:33-50"""
    c_transformer = CTransformer(transformer.channel_size, transformer.raw_channels_per_state,
                                 transformer.num_of_controls_channels, transformer.num_previous_states,
                                 transformer.num_rewards, transformer.policy_dist_count)
    for b in transformer.board_space:
        index = transformer.channel_size * b.channel_id + b.y_idx * transformer.num_rows + b.x_idx
        c_transformer.add_board_base(b.base_indx, index)
    for c in transformer.control_space:
        c_transformer.add_control_base(c.base_indx, c.channel_id, c.value)
    return c_transformer


def _planes_view(ptr, buf_count):
    """Zero-copy float32 view of the engine-owned planes buffer (common.cpp:200-212)."""
    return np.ctypeslib.as_array(ptr, shape=(buf_count,))


class _CSupervisor(object):
    """ggpzero_interface.Supervisor (supervisor_impl.cpp:146-237) over gz_supervisor_*."""

    def __init__(self, sm, c_transformer, batch_size, identifier, seed=0, per_pool_unique_states=False):
        self.lib = _native.engine_lib()
        self.sm = sm
        self.c_transformer = c_transformer
        self.handle = self.lib.gz_supervisor_create(sm_to_ptr(sm), c_transformer.handle, batch_size,
                                                    identifier.encode(), seed, int(per_pool_unique_states))
        if not self.handle:
            raise RuntimeError(_native.engine_error())
        self._keep = None

    def start_self_play(self, num_workers, conf_dict):
        c = _native.make_selfplay_config(conf_dict)
        if self.lib.gz_supervisor_start_self_play(self.handle, num_workers, ctypes.byref(c)) != 0:
            raise RuntimeError(_native.engine_error())

    def poll(self, predict_count, arrays):
        self._keep, ptrs = _as_float_arrays(arrays)
        count = ctypes.c_int(0)
        ptr = self.lib.gz_supervisor_poll(self.handle, predict_count, ptrs, len(arrays), ctypes.byref(count))
        if count.value < 0:
            raise RuntimeError("poll failed: %s" % _native.engine_error())
        if count.value == 0:
            return None
        return _planes_view(ptr, count.value)

    def fetch_samples(self):
        s = _native.take_string(self.lib.gz_supervisor_fetch_samples(self.handle))
        return json.loads(s) if s else None

    def cancel(self):
        if self.lib.gz_supervisor_cancel(self.handle) != 0:
            raise RuntimeError(_native.engine_error())

    def add_unique_state(self, state_words):
        s = np.ascontiguousarray(state_words, dtype=np.uint64)
        self.lib.gz_supervisor_add_unique_state(self.handle, s.ctypes.data_as(_U64P))

    def clear_unique_states(self):
        self.lib.gz_supervisor_clear_unique_states(self.handle)

    def set_sample_interval(self, polls):
        self.lib.gz_supervisor_set_sample_interval(self.handle, polls)

    def stats(self):
        st = _native.GzPoolStats()
        self.lib.gz_supervisor_stats(self.handle, ctypes.byref(st))
        return st.as_dict()

    def __del__(self):
        try:
            if self.handle:
                self.lib.gz_supervisor_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class _CPlayer(object):
    """ggpzero_interface.Player (player_impl.cpp:116-201) over gz_player_*."""

    def __init__(self, sm, c_transformer, conf_dict, seed=0):
        self.lib = _native.engine_lib()
        self.sm = sm
        self.c_transformer = c_transformer
        c = _native.make_puct_config(conf_dict)
        self.handle = self.lib.gz_player_create(sm_to_ptr(sm), c_transformer.handle, ctypes.byref(c), seed)
        if not self.handle:
            raise RuntimeError(_native.engine_error())
        self._keep = None
        self._state = None

    def player_reset(self, game_depth=0):
        self.lib.gz_player_reset(self.handle, game_depth)

    def player_apply_move(self, joint_move):
        jm = (ctypes.c_int * self.sm.role_count)(*joint_move)
        self.lib.gz_player_apply_move(self.handle, jm)

    def player_move(self, state_words, iterations, end_time=-1.0):
        self._state = np.ascontiguousarray(state_words, dtype=np.uint64)
        self.lib.gz_player_move(self.handle, self._state.ctypes.data_as(_U64P), iterations, end_time)

    def player_get_move(self, lead_role_index):
        legal, nodes, prob = ctypes.c_int(), ctypes.c_int(), ctypes.c_float()
        self.lib.gz_player_get_move(self.handle, lead_role_index, ctypes.byref(legal), ctypes.byref(prob),
                                    ctypes.byref(nodes))
        return legal.value, prob.value, nodes.value

    def player_update_config(self, think_time, converged_visits, verbose):
        self.lib.gz_player_update_config(self.handle, think_time, converged_visits, int(verbose))

    def player_balance_moves(self, max_count):
        self.lib.gz_player_balance_moves(self.handle, max_count)

    def player_tree_debug(self, max_count):
        s = _native.take_string(self.lib.gz_player_tree_debug(self.handle, max_count))
        return json.loads(s) if s else []

    def root_children(self):
        cap = 4096
        moves = (ctypes.c_int * cap)()
        trav = (ctypes.c_uint32 * cap)()
        probs = (ctypes.c_float * cap)()
        n = self.lib.gz_player_root_children(self.handle, moves, trav, probs, cap)
        return [(moves[i], trav[i], probs[i]) for i in range(min(n, cap))]

    def poll(self, predict_count, arrays):
        # the Player stores these pointers until the next poll (player.cpp:160-168): keep them alive
        self._keep, ptrs = _as_float_arrays(arrays)
        count = ctypes.c_int(0)
        ptr = self.lib.gz_player_poll(self.handle, predict_count, ptrs, len(arrays), ctypes.byref(count))
        if count.value < 0:
            raise RuntimeError("poll failed: %s" % _native.engine_error())
        if count.value == 0:
            return None
        return _planes_view(ptr, count.value)

    def __del__(self):
        try:
            if self.handle:
                self.lib.gz_player_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class PollerBase(object):
    """cppinterface.py:53-153"""
    POLL_AGAIN = "poll_again"

    def __init__(self, sm, nn, batch_size=1024, sleep_between_poll=-1):
        self.sm = sm
        self.nn = nn
        self.batch_size = batch_size
        self.sleep_between_poll = sleep_between_poll
        self.poll_last = None
        self.reset_stats()

    def _get_poller(self):
        raise NotImplementedError

    def reset_stats(self):
        self.num_predictions_calls = 0
        self.total_predictions = 0
        self.acc_time_polling = 0
        self.acc_time_prediction = 0

    def poll(self, do_stats=False):
        """POLL_AGAIN is returned to indicate poll() must be called again."""
        transformer = self.nn.gdl_bases_transformer
        expect_num_arrays = len(transformer.policy_dist_count) + 1
        if self.poll_last is None:
            dummy = np.zeros(0, dtype=np.float32)
            arrays = [dummy for _ in range(expect_num_arrays)]
        else:
            arrays = list(self.poll_last)
        assert len(arrays) == expect_num_arrays

        if do_stats:
            s0 = time.time()
        pred_array = self._get_poller().poll(len(arrays[0]), arrays)
        if pred_array is None:
            self.poll_last = None
            return
        if do_stats:
            s1 = time.time()

        t = transformer
        num_predictions = len(pred_array) // (t.num_channels * t.channel_size)
        assert num_predictions <= self.batch_size
        pred_array = pred_array.reshape(num_predictions, t.num_channels, t.num_cols, t.num_rows)
        self.poll_last = self.nn.get_model().predict_on_batch(pred_array)

        if do_stats:
            s2 = time.time()
            self.num_predictions_calls += 1
            self.total_predictions += num_predictions
            self.acc_time_polling += s1 - s0
            self.acc_time_prediction += s2 - s1
        return self.POLL_AGAIN

    def poll_loop(self, cb=None, do_stats=False, cb_every_n=100):
        count = 1
        while self.poll(do_stats=do_stats) == self.POLL_AGAIN:
            if count % cb_every_n == 0 and cb is not None and cb():
                break
            count += 1
            if self.sleep_between_poll > 0:
                time.sleep(self.sleep_between_poll)

    def update_nn(self, nn):
        self.nn = nn

    def dump_stats(self):
        print("num of prediction calls", self.num_predictions_calls)
        print("predictions", self.total_predictions)
        print("acc_time_polling", self.acc_time_polling)
        print("acc_time_prediction", self.acc_time_prediction)


class PlayPoller(PollerBase):
    """cppinterface.py:156-182"""

    def __init__(self, sm, nn, conf, seed=0):
        assert isinstance(conf, confs.PUCTEvaluatorConfig)
        super(PlayPoller, self).__init__(sm, nn, batch_size=conf.batch_size)
        self.c_transformer = create_c_transformer(nn.gdl_bases_transformer)
        self.c_player = _CPlayer(sm, self.c_transformer, conf, seed=seed)
        for name in "reset apply_move move get_move update_config balance_moves tree_debug".split():
            name = "player_" + name
            setattr(self, name, getattr(self.c_player, name))

    def _get_poller(self):
        return self.c_player


class Supervisor(PollerBase):
    """cppinterface.py:185-226.  Extra keyword arguments: seed (global RNG seed) and
    per_pool_unique_states (deterministic duplicate filter)."""

    def __init__(self, sm, nn, batch_size=1024, sleep_between_poll=-1, workers=None, identifier="",
                 seed=0, per_pool_unique_states=False):
        transformer = nn.gdl_bases_transformer
        self.c_transformer = create_c_transformer(transformer)
        self.c_supervisor = _CSupervisor(sm, self.c_transformer, batch_size, identifier, seed=seed,
                                         per_pool_unique_states=per_pool_unique_states)
        self.workers = workers
        super(Supervisor, self).__init__(sm, nn, batch_size=batch_size, sleep_between_poll=sleep_between_poll)

    def _get_poller(self):
        return self.c_supervisor

    def start_self_play(self, conf, num_workers):
        assert isinstance(conf, confs.SelfPlayConfig)
        return self.c_supervisor.start_self_play(num_workers, conf)

    def fetch_samples(self):
        res = self.c_supervisor.fetch_samples()
        if res:
            return [datadesc.Sample(**d) for d in res]
        return []

    def add_unique_state(self, s):
        return  # no-op in the reference too (cppinterface.py:218-219)

    def clear_unique_states(self):
        self.c_supervisor.clear_unique_states()

    def cancel(self):
        """Bounded teardown (build extension), callable from another thread: the pools stop at their
        games' next playout and poll() -- one in progress included -- returns None from then on, so
        poll_loop() ends."""
        self.c_supervisor.cancel()

    def stats(self):
        return self.c_supervisor.stats()
