"""ORACLE (test infrastructure only) -- pure-Python restatement of the GDL rule sheets for the
native state machines (galvanise_zero_amd/csrc/engine/games.cpp).

Breakthrough N x N: data/rulesheets/breakthrough.kif (N=8, base term cellHolds) and
breakthroughSmall.kif (N=6, base term cell):
  * legal (kif LEGAL section): the role in control moves a piece one row forward (white +1,
    black -1) onto an empty cell, or diagonally onto a cell not holding its own piece; the other
    role plays noop;
  * next (kif NEXT section): the moved piece lands on (x2,y2), every other cell persists unless it
    is the source or destination; control alternates;
  * terminal / goal: whiteWin = a white piece on row N or no black piece (MG's bugfix); blackWin
    symmetric on row 1; goal 100 / 0.
Legality is evaluated rule by rule over the whole input action list (an independent formulation
of the engine's bitboard move generator).  Base and action orders are the build's canonical ones
(ggplib's are unpinned): base cell(x,y,r) = ((x-1)*N+(y-1))*2+r, control(white)=2N^2,
control(black)=2N^2+1; actions: noop, forward (x-major, y1), right diagonals (y1-major, x1),
left diagonals (y1-major, x1).
"""


class Breakthrough(object):
    def __init__(self, n=8, cell_term="cellHolds", game="breakthrough"):
        self.N = n
        self.game = game
        self.cell_term = cell_term
        self.role_count = 2
        self.num_bases = 2 * n * n + 2
        self.actions = [self._action_list(r) for r in range(2)]
        init = 0
        for x in range(1, n + 1):
            for y in (1, 2):
                init |= 1 << self.cell(x, y, 0)
            for y in (n - 1, n):
                init |= 1 << self.cell(x, y, 1)
        init |= 1 << (2 * n * n)
        self.initial_state = init

    def cell(self, x, y, r):
        return ((x - 1) * self.N + (y - 1)) * 2 + r

    def base_name(self, i):
        n = self.N
        if i >= 2 * n * n:
            return "(control %s)" % ("white" if i == 2 * n * n else "black")
        c, r = divmod(i, 2)
        x, y = divmod(c, n)
        return "(%s %d %d %s)" % (self.cell_term, x + 1, y + 1, "white" if r == 0 else "black")

    def _action_list(self, role):
        n = self.N
        acts = [None]                      # noop
        ys = [(y, y + 1) for y in range(1, n)] if role == 0 else [(y, y - 1) for y in range(2, n + 1)]
        for x in range(1, n + 1):
            for y1, y2 in ys:
                acts.append(("fwd", x, y1, x, y2))
        for y1, y2 in ys:
            for x1 in range(1, n):
                acts.append(("diag", x1, y1, x1 + 1, y2))
        for y1, y2 in ys:
            for x1 in range(2, n + 1):
                acts.append(("diag", x1, y1, x1 - 1, y2))
        return acts

    def action_count(self, role):
        return len(self.actions[role])

    def _holds(self, s, x, y, r):
        return (s >> self.cell(x, y, r)) & 1

    def control(self, s):
        return 0 if (s >> (2 * self.N * self.N)) & 1 else 1

    def legal(self, s, role):
        if self.control(s) != role:
            return [0]
        out = []
        for a, act in enumerate(self.actions[role]):
            if act is None:
                continue
            kind, x1, y1, x2, y2 = act
            if not self._holds(s, x1, y1, role):
                continue
            if kind == "fwd":
                if not self._holds(s, x2, y2, 0) and not self._holds(s, x2, y2, 1):
                    out.append(a)
            elif not self._holds(s, x2, y2, role):
                out.append(a)
        return out

    def _wins(self, s):
        n = self.N
        white_cells = any(self._holds(s, x, y, 0) for x in range(1, n + 1) for y in range(1, n + 1))
        black_cells = any(self._holds(s, x, y, 1) for x in range(1, n + 1) for y in range(1, n + 1))
        white_win = any(self._holds(s, x, n, 0) for x in range(1, n + 1)) or not black_cells
        black_win = any(self._holds(s, x, 1, 1) for x in range(1, n + 1)) or not white_cells
        return white_win, black_win

    def is_terminal(self, s):
        w, b = self._wins(s)
        return w or b

    def goal(self, s, role):
        w, b = self._wins(s)
        return 100 if (w if role == 0 else b) else 0

    def next_state(self, s, joint):
        n = self.N
        out = 0
        moves = [self.actions[r][joint[r]] for r in range(2)]
        for r, m in enumerate(moves):
            if m is not None:
                out |= 1 << self.cell(m[3], m[4], r)
        for x in range(1, n + 1):
            for y in range(1, n + 1):
                for r in range(2):
                    if not self._holds(s, x, y, r):
                        continue
                    keep = True
                    for m in moves:
                        if m is not None and ((m[1], m[2]) == (x, y) or (m[3], m[4]) == (x, y)):
                            keep = False
                    if keep:
                        out |= 1 << self.cell(x, y, r)
        out |= 1 << (2 * n * n + (1 - self.control(s)))
        return out

    def legal_to_move(self, role, a):
        act = self.actions[role][a]
        if act is None:
            return "noop"
        return "(move %d %d %d %d)" % act[1:]


def make(game):
    if game == "breakthrough":
        return Breakthrough(8, "cellHolds", "breakthrough")
    if game == "breakthroughSmall":
        return Breakthrough(6, "cell", "breakthroughSmall")
    raise KeyError(game)


def state_to_words(s, num_bases):
    nw = (num_bases + 63) // 64
    return [(s >> (64 * i)) & ((1 << 64) - 1) for i in range(nw)]


def words_to_state(words):
    s = 0
    for i, w in enumerate(words):
        s |= int(w) << (64 * i)
    return s
