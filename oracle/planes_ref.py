"""ORACLE (test infrastructure only) -- restatement of the state -> input planes transform.

* geometry: reference src/ggpzero/nn/bases.py:168-240 (create_board_space / create_control_space)
  with the per-game descriptions of src/ggpzero/defs/gamedesc.py:142-175;
* buffer offsets: cppinterface.py:42-48 (channel_size*channel_id + y_idx*num_rows + x_idx);
* planes: gdltransformer.cpp:22-52 toChannels (zero, board bits of the state, board bits of each
  previous state all in slot 1 -- the reference never advances `count` --, control flood fill).
"""
import numpy as np

# Per-game descriptions restated from src/ggpzero/defs/gamedesc.py (helpers :116-134):
#   x/y coords (gamedesc GameDesc.x_cords / y_cords), board channels as
#   (base term, x term idx, y term idx, piece term idx or None, pieces) (BoardChannels / BoardTerm),
#   control channels as [[(arg terms, value), ...], ...] (ControlChannel / ControlBase).
_C8 = [str(i) for i in range(1, 9)]


def _binary(base, a, b):            # gamedesc.py:120-122
    return [((base, a), 0), ((base, b), 1)]


GAME_DESCS = {
    # gamedesc.py:142-150
    "breakthrough": dict(x=_C8, y=_C8, board=[("cellHolds", 1, 2, 3, ["white", "black"])],
                         controls=[_binary("control", "black", "white")]),
    # gamedesc.py:169-175
    "breakthroughSmall": dict(x=_C8[:6], y=_C8[:6], board=[("cell", 1, 2, 3, ["white", "black"])],
                              controls=[_binary("control", "white", "black")]),
    # gamedesc.py:152-160
    "reversi": dict(x=_C8, y=_C8, board=[("cell", 1, 2, 3, ["black", "red"])],
                    controls=[_binary("control", "black", "red")]),
    # gamedesc.py:309-318
    "hexLG13": dict(x=list("abcdefghijklm"), y=[str(i) for i in range(1, 14)],
                    board=[("cell", 1, 2, 3, ["black", "white"])],
                    controls=[_binary("control", "black", "white")]),
    # gamedesc.py:214-232 (simple_control = one base, value 1)
    "amazons_10x10": dict(x=[str(i) for i in range(1, 11)], y=[str(i) for i in range(1, 11)],
                          board=[("justMoved", 1, 2, None, None), ("cell", 1, 2, 3, ["white", "black", "arrow"])],
                          controls=[[(("turn", "black", "move"), 1)], [(("turn", "black", "fire"), 1)],
                                    [(("turn", "white", "move"), 1)], [(("turn", "white", "fire"), 1)]]),
}


class Planes(object):
    def __init__(self, game, base_names, num_prev_states=1):
        d = GAME_DESCS[game]
        self.num_prev_states = num_prev_states
        terms = [n.strip("()").split() for n in base_names]
        self.W = len(d["x"])               # num_rows = len(x_cords)   (bases.py:104-121)
        self.H = len(d["y"])               # num_cols = len(y_cords)
        self.channel_size = self.W * self.H
        board, mapping, used = [], {}, set()
        # bases.py:168-213 create_board_space: first board channel whose base term matches; the
        # channel key is (base term, matched piece terms), numbered in first-seen base order
        for idx, t in enumerate(terms):
            bc = next((b for b in d["board"] if b[0] == t[0]), None)
            if bc is None:
                continue
            base, xi, yi, pi, pieces = bc
            if pi is not None and t[pi] not in pieces:
                continue
            key = (t[0],) if pi is None else (t[0], t[pi])
            mapping.setdefault(key, len(mapping))
            x = d["x"].index(t[xi])
            y = d["y"].index(t[yi])
            # cppinterface.py:44: channel_size * channel_id + y_idx * num_rows + x_idx
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
