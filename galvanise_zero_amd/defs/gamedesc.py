"""Per-game board / control channel descriptions (reference src/ggpzero/defs/gamedesc.py:5-150):
which GDL bases become board planes and which flood-fill a control plane, and with what value."""
import attr


@attr.s
class ControlBase(object):
    arg_terms = attr.ib(factory=list)
    value = attr.ib(default=1)


@attr.s
class ControlChannel(object):
    control_bases = attr.ib(factory=list)


@attr.s
class BoardTerm(object):
    term_idx = attr.ib(default=3)
    terms = attr.ib(factory=list)


@attr.s
class BoardChannels(object):
    base_term = attr.ib(default="cell")
    x_term_idx = attr.ib(default=1)
    y_term_idx = attr.ib(default=2)
    board_terms = attr.ib(factory=list)


@attr.s
class GameDesc(object):
    game = attr.ib(default="checkers")
    x_cords = attr.ib(factory=list)
    y_cords = attr.ib(factory=list)
    board_channels = attr.ib(factory=list)
    control_channels = attr.ib(factory=list)


def simple_control(*terms):
    return ControlChannel([ControlBase(list(terms), 1)])


def binary_control(base_term, a_term, b_term):
    return ControlChannel([ControlBase([base_term, a_term], 0), ControlBase([base_term, b_term], 1)])


def simple_board_channels(base, pieces):
    return BoardChannels(base, 1, 2, [BoardTerm(3, pieces)])


def _cords(n):
    return [str(i) for i in range(1, n + 1)]


class Games(object):
    def breakthrough(self):
        # control polarity: black -> 0, white -> 1 (gamedesc.py:144)
        return GameDesc("breakthrough", _cords(8), _cords(8),
                        [simple_board_channels("cellHolds", ["white", "black"])],
                        [binary_control("control", "black", "white")])

    def breakthroughSmall(self):
        # control polarity reversed: white -> 0, black -> 1 (gamedesc.py:173)
        return GameDesc("breakthroughSmall", _cords(6), _cords(6),
                        [simple_board_channels("cell", ["white", "black"])],
                        [binary_control("control", "white", "black")])

    def reversi(self):
        # gamedesc.py:152-160: cell {black, red}; control black -> 0, red -> 1
        return GameDesc("reversi", _cords(8), _cords(8),
                        [simple_board_channels("cell", ["black", "red"])],
                        [binary_control("control", "black", "red")])

    def hexLG13(self):
        # gamedesc.py:309-318: x = row letters a..m, y = numbers 1..13; control black -> 0, white -> 1
        return GameDesc("hex", list("abcdefghijklm"), _cords(13),
                        [simple_board_channels("cell", ["black", "white"])],
                        [binary_control("control", "black", "white")])

    def amazons_10x10(self):
        # gamedesc.py:216-232: justMoved plane + cell {white, black, arrow}; four turn planes
        controls = [simple_control("turn", "black", "move"), simple_control("turn", "black", "fire"),
                    simple_control("turn", "white", "move"), simple_control("turn", "white", "fire")]
        return GameDesc("amazons_10x10", _cords(10), _cords(10),
                        [BoardChannels("justMoved", 1, 2),
                         simple_board_channels("cell", ["white", "black", "arrow"])],
                        controls)

    def bt_7(self):
        return GameDesc("breakthrough", _cords(7), _cords(7),
                        [simple_board_channels("cellHolds", ["white", "black"])],
                        [binary_control("control", "black", "white")])
