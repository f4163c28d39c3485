"""Native game state machines (stand-in for ggplib's StateMachine + lookup.by_name(game).get_sm(),
used by the reference at cppinterface.py:12-16 and nn/manager.py:78)."""
import ctypes

import numpy as np

from ._native import engine_error, engine_lib

_U64P = ctypes.POINTER(ctypes.c_uint64)


def _u64(a):
    return a.ctypes.data_as(_U64P)


class StateMachine(object):
    def __init__(self, game):
        self.lib = engine_lib()
        self.game = game
        self.handle = self.lib.gz_sm_create(game.encode())
        if not self.handle:
            raise ValueError(engine_error())
        self.role_count = self.lib.gz_sm_role_count(self.handle)
        self.num_bases = self.lib.gz_sm_num_bases(self.handle)
        self.num_words = self.lib.gz_sm_num_words(self.handle)

    def _str(self, fn, *args):
        buf = ctypes.create_string_buffer(256)
        fn(self.handle, *args, buf, 256)
        return buf.value.decode()

    def base_name(self, i):
        return self._str(self.lib.gz_sm_base_name, i)

    def role_name(self, r):
        return self._str(self.lib.gz_sm_role_name, r)

    def legal_to_move(self, role, action):
        return self._str(self.lib.gz_sm_legal_to_move, role, action)

    def action_count(self, role):
        return self.lib.gz_sm_action_count(self.handle, role)

    def new_base_state(self):
        return np.zeros(self.num_words, dtype=np.uint64)

    def get_initial_state(self):
        s = self.new_base_state()
        self.lib.gz_sm_initial_state(self.handle, _u64(s))
        return s

    def update_bases(self, state):
        self._state = np.ascontiguousarray(state, dtype=np.uint64)
        self.lib.gz_sm_update_bases(self.handle, _u64(self._state))

    def get_legal_state(self, role):
        n = self.lib.gz_sm_legal_count(self.handle, role)
        return [self.lib.gz_sm_legal(self.handle, role, i) for i in range(n)]

    def is_terminal(self):
        return bool(self.lib.gz_sm_is_terminal(self.handle))

    def get_goal_value(self, role):
        return self.lib.gz_sm_goal_value(self.handle, role)

    def next_state(self, joint_move):
        out = self.new_base_state()
        jm = (ctypes.c_int * self.role_count)(*joint_move)
        self.lib.gz_sm_next_state(self.handle, jm, _u64(out))
        return out

    def bits(self, state):
        """word array -> tuple of 0/1 over the bases (the Sample 'state' encoding)."""
        words = np.ascontiguousarray(state, dtype=np.uint64)
        return tuple(int((int(words[i >> 6]) >> (i & 63)) & 1) for i in range(self.num_bases))

    def from_bits(self, bits):
        out = self.new_base_state()
        for i, b in enumerate(bits):
            if b:
                out[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
        return out

    def __del__(self):
        try:
            if self.handle:
                self.lib.gz_sm_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def get_sm(game):
    return StateMachine(game)
