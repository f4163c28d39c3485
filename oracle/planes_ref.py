"""ORACLE (test infrastructure only) -- restatement of the state -> input planes transform.

* geometry: reference src/ggpzero/nn/bases.py:168-240 (create_board_space / create_control_space)
  with the per-game descriptions of src/ggpzero/defs/gamedesc.py:142-175;
* buffer offsets: cppinterface.py:42-48 (channel_size*channel_id + y_idx*num_rows + x_idx);
* planes: gdltransformer.cpp:22-52 toChannels (zero, board bits of the state, board bits of each
  previous state all in slot 1 -- the reference never advances `count` --, control flood fill).
"""
import numpy as np

# gamedesc.py:142-150, 169-175: (board base term, piece terms, x/y term idx, piece term idx,
# coords, control channels [[(args, value), ...], ...])
GAME_DESCS = {
    "breakthrough": dict(base_term="cellHolds", pieces=["white", "black"], x_idx=1, y_idx=2, piece_idx=3,
                         coords=[str(i) for i in range(1, 9)],
                         controls=[[(("control", "black"), 0), (("control", "white"), 1)]]),
    "breakthroughSmall": dict(base_term="cell", pieces=["white", "black"], x_idx=1, y_idx=2, piece_idx=3,
                              coords=[str(i) for i in range(1, 7)],
                              controls=[[(("control", "white"), 0), (("control", "black"), 1)]]),
}


class Planes(object):
    def __init__(self, game, base_names, num_prev_states=1):
        d = GAME_DESCS[game]
        self.num_prev_states = num_prev_states
        terms = [n.strip("()").split() for n in base_names]
        self.W = len(d["coords"])          # num_rows = len(x_cords)
        self.H = len(d["coords"])          # num_cols = len(y_cords)
        self.channel_size = self.W * self.H
        board, mapping, used = [], {}, set()
        for idx, t in enumerate(terms):
            if t[0] != d["base_term"] or t[d["piece_idx"]] not in d["pieces"]:
                continue
            key = (t[0], t[d["piece_idx"]])
            mapping.setdefault(key, len(mapping))
            x = d["coords"].index(t[d["x_idx"]])
            y = d["coords"].index(t[d["y_idx"]])
            board.append((idx, self.channel_size * mapping[key] + y * self.W + x))
            used.add(idx)
        self.board = board
        self.channels_per_state = len(mapping)
        self.control = []
        for cid, cc in enumerate(d["controls"]):
            for idx, t in enumerate(terms):
                for args, value in cc:
                    if tuple(t) == args:
                        self.control.append((idx, cid, np.float32(value)))
                        used.add(idx)
                        break
        self.num_control_channels = len(d["controls"])
        self.num_channels = self.channels_per_state * (num_prev_states + 1) + self.num_control_channels
        self.total_size = self.channel_size * self.num_channels

    def to_channels(self, state, prev_states=()):
        """state / prev_states: python ints (bit i = base i)."""
        buf = np.zeros(self.total_size, dtype=np.float32)
        for idx, off in self.board:
            if (state >> idx) & 1:
                buf[off] = 1.0
        count = 1
        for p in list(prev_states)[:self.num_prev_states]:
            base = self.channels_per_state * self.channel_size * count
            for idx, off in self.board:
                if (p >> idx) & 1:
                    buf[base + off] = 1.0
        start = self.channel_size * self.channels_per_state * (self.num_prev_states + 1)
        for idx, cid, value in self.control:
            if (state >> idx) & 1:
                buf[start + cid * self.channel_size:start + (cid + 1) * self.channel_size] = value
        return buf

    def hash_mask(self):
        m = 0
        for idx, _ in self.board:
            m |= 1 << idx
        for idx, _, _ in self.control:
            m |= 1 << idx
        return m
