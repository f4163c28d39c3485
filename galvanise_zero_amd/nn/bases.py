"""Input-plane geometry: restates the Python GdlBasesTransformer (reference src/ggpzero/nn/bases.py:
63-287) over a native state machine's base names instead of a ggplib game model.

num_rows = len(x_cords) = W, num_cols = len(y_cords) = H, planes are [C][H][W]; board bases map to
(channel_id, y_idx, x_idx); control bases flood-fill channel `raw_channels_per_state*(prev+1) +
channel_id` with their value.
"""
import numpy as np

from ..defs import datadesc, gamedesc


def parse_terms(base_name):
    """'(cellHolds 1 2 white)' -> ['cellHolds', '1', '2', 'white']"""
    s = base_name.strip()
    if s.startswith("("):
        s = s[1:-1]
    return s.split()


class BaseToBoardSpace(object):
    def __init__(self, base_indx, channel_id, x_idx, y_idx):
        self.base_indx, self.channel_id, self.x_idx, self.y_idx = base_indx, channel_id, x_idx, y_idx


class BaseToChannelSpace(object):
    def __init__(self, base_indx, channel_id, value):
        self.base_indx, self.channel_id, self.value = base_indx, channel_id, value


class GdlBasesTransformer(object):
    def __init__(self, sm, generation_descr, game_desc=None):
        assert isinstance(generation_descr, datadesc.GenerationDescription)
        self.sm = sm
        self.game = sm.game
        if game_desc is None:
            game_desc = getattr(gamedesc.Games(), sm.game)()
        self.game_desc = game_desc
        self.role_count = sm.role_count
        assert generation_descr.multiple_policy_heads
        self.policy_dist_count = [sm.action_count(r) for r in range(sm.role_count)]
        self.final_score_count = sm.role_count
        self.channel_last = generation_descr.channel_last
        self.num_previous_states = generation_descr.num_previous_states
        self.num_rewards = 3 if generation_descr.draw_head else 2
        self.init_spaces()

    @property
    def x_cords(self):
        return self.game_desc.x_cords

    @property
    def y_cords(self):
        return self.game_desc.y_cords

    @property
    def num_rows(self):
        return len(self.x_cords)

    @property
    def num_cols(self):
        return len(self.y_cords)

    @property
    def channel_size(self):
        return self.num_cols * self.num_rows

    @property
    def num_bases(self):
        return self.sm.num_bases

    @property
    def num_channels(self):
        return self.num_of_controls_channels + self.raw_channels_per_state * (self.num_previous_states + 1)

    def init_spaces(self):
        terms = [parse_terms(self.sm.base_name(i)) for i in range(self.sm.num_bases)]
        used = [False] * len(terms)
        # bases.py:168-218
        self.board_space = []
        channel_mapping = {}
        for idx, t in enumerate(terms):
            bc = None
            for cand in self.game_desc.board_channels:
                if t[0] == cand.base_term:
                    bc = cand
                    break
            if bc is None:
                continue
            matched = [t[bt.term_idx] for bt in bc.board_terms if t[bt.term_idx] in bt.terms]
            if len(matched) != len(bc.board_terms):
                continue
            key = tuple([t[0]] + matched)
            if key not in channel_mapping:
                channel_mapping[key] = len(channel_mapping)
            x_idx = self.game_desc.x_cords.index(t[bc.x_term_idx])
            y_idx = self.game_desc.y_cords.index(t[bc.y_term_idx])
            self.board_space.append(BaseToBoardSpace(idx, channel_mapping[key], x_idx, y_idx))
            used[idx] = True
        self.raw_channels_per_state = max(b.channel_id for b in self.board_space) + 1
        # bases.py:220-240
        self.control_space = []
        for channel_id, cc in enumerate(self.game_desc.control_channels):
            for idx, t in enumerate(terms):
                for cb in cc.control_bases:
                    if tuple(t) == tuple(cb.arg_terms):
                        assert not used[idx]
                        self.control_space.append(BaseToChannelSpace(idx, channel_id, cb.value))
                        used[idx] = True
                        break
        self.num_of_controls_channels = len(self.game_desc.control_channels)
        self.num_unhandled_states = used.count(False)

    def state_to_channels(self, state, prev_states=None):
        """bases.py:242-287: state is a sequence of 0/1 over the bases."""
        prev_states = prev_states or []
        assert len(prev_states) <= self.num_previous_states
        ch = np.zeros((self.num_channels, self.num_cols, self.num_rows), dtype=np.float32)
        for b in self.board_space:
            if state[b.base_indx]:
                ch[b.channel_id, b.y_idx, b.x_idx] = 1
        incr = self.raw_channels_per_state
        for ii in range(self.num_previous_states):
            if ii < len(prev_states):
                for b in self.board_space:
                    if prev_states[ii][b.base_indx]:
                        ch[b.channel_id + incr, b.y_idx, b.x_idx] = 1
            incr += self.raw_channels_per_state
        for c in self.control_space:
            if state[c.base_indx]:
                ch[c.channel_id + incr] += c.value
        if self.channel_last:
            ch = np.rollaxis(np.rollaxis(ch, -1), -1)
        return ch

    def policy_to_array(self, policy, role_index):
        array = np.zeros(self.policy_dist_count[role_index], dtype=np.float32)
        for idx, prob in policy:
            array[idx] = prob
        return array

    def value_to_array(self, values):
        assert len(values) == self.role_count
        return np.array(values, dtype=np.float32)
