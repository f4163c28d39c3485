"""ORACLE (test infrastructure only) -- pure-Python restatement of the GDL rule sheets for the
native state machines (galvanise_zero_amd/csrc/engine/games.cpp, games_more.cpp): breakthrough,
breakthroughSmall, reversi, hexLG13, amazons_10x10 (classes below cite their rule sheets).

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


class Reversi(object):
    """data/rulesheets/reversi.kif, rule by rule: hasOtherColorInDir (recursive run test),
    playerCanMoveAt, legal (noop when not in control or when no move), affected (flip propagation
    from the placed disc outwards, per direction), terminal (neither role can move), goal by
    pieceCount (100 / 0, 50 each when equal).  Roles black (0), red (1); base
    cell(x,y,c) = ((x-1)*8+(y-1))*2+c, control black 128, red 129; action 1+(x-1)*8+(y-1)."""
    N = 8
    DIRS = {"n": (0, 1), "s": (0, -1), "e": (1, 0), "w": (-1, 0),
            "nw": (-1, 1), "ne": (1, 1), "se": (1, -1), "sw": (-1, -1)}

    def __init__(self):
        self.game = "reversi"
        self.role_count = 2
        self.num_bases = 2 * 64 + 2
        s = 0
        for (x, y, c) in ((4, 4, 0), (4, 5, 1), (5, 4, 1), (5, 5, 0)):
            s |= 1 << self.cell(x, y, c)
        self.initial_state = s | (1 << 128)

    def cell(self, x, y, c):
        return ((x - 1) * 8 + (y - 1)) * 2 + c

    def base_name(self, i):
        if i >= 128:
            return "(control %s)" % ("black" if i == 128 else "red")
        c, r = divmod(i, 2)
        return "(cell %d %d %s)" % (c // 8 + 1, c % 8 + 1, "black" if r == 0 else "red")

    def action_count(self, role):
        return 65

    def legal_to_move(self, role, a):
        return "noop" if a == 0 else "(move %d %d)" % ((a - 1) // 8 + 1, (a - 1) % 8 + 1)

    def _color(self, s, x, y):
        for c in (0, 1):
            if (s >> self.cell(x, y, c)) & 1:
                return c
        return None

    def _next_in_dir(self, x, y, d):
        dx, dy = self.DIRS[d]
        x2, y2 = x + dx, y + dy
        return (x2, y2) if 1 <= x2 <= 8 and 1 <= y2 <= 8 else None

    def _has_other_color_in_dir(self, s, x, y, d):
        c = self._color(s, x, y)
        nxt = self._next_in_dir(x, y, d)
        if c is None or nxt is None:
            return False
        c2 = self._color(s, *nxt)
        if c2 is None:
            return False
        return c2 != c or self._has_other_color_in_dir(s, nxt[0], nxt[1], d)

    def _can_move_at(self, s, c, x, y):
        if self._color(s, x, y) is not None:
            return False
        for d in self.DIRS:
            nxt = self._next_in_dir(x, y, d)
            if nxt and self._color(s, *nxt) == 1 - c and self._has_other_color_in_dir(s, nxt[0], nxt[1], d):
                return True
        return False

    def _can_move(self, s, c):
        return any(self._can_move_at(s, c, x, y) for x in range(1, 9) for y in range(1, 9))

    def control(self, s):
        return 0 if (s >> 128) & 1 else 1

    def legal(self, s, role):
        if self.control(s) != role or not self._can_move(s, role):
            return [0]
        return [1 + (x - 1) * 8 + (y - 1) for x in range(1, 9) for y in range(1, 9)
                if self._can_move_at(s, role, x, y)]

    def is_terminal(self, s):
        return not self._can_move(s, 0) and not self._can_move(s, 1)

    def goal(self, s, role):
        cnt = [0, 0]
        for x in range(1, 9):
            for y in range(1, 9):
                c = self._color(s, x, y)
                if c is not None:
                    cnt[c] += 1
        if cnt[0] == cnt[1]:
            return 50
        return 100 if cnt[role] > cnt[1 - role] else 0

    def next_state(self, s, joint):
        mover = self.control(s)
        a = joint[mover]
        affected = set()
        if a:
            x1, y1 = (a - 1) // 8 + 1, (a - 1) % 8 + 1
            for d in self.DIRS:
                nxt = self._next_in_dir(x1, y1, d)
                # affected(x2,y2,dir,other) then propagated while hasOtherColorInDir
                while nxt and self._color(s, *nxt) == 1 - mover and \
                        self._has_other_color_in_dir(s, nxt[0], nxt[1], d):
                    affected.add(nxt)
                    nxt = self._next_in_dir(nxt[0], nxt[1], d)
        out = 0
        for x in range(1, 9):
            for y in range(1, 9):
                c = self._color(s, x, y)
                if a and (x, y) == ((a - 1) // 8 + 1, (a - 1) % 8 + 1):
                    c = mover
                elif (x, y) in affected:
                    c = mover
                if c is not None:
                    out |= 1 << self.cell(x, y, c)
        return out | (1 << (128 + (1 - mover)))


class HexLG13(object):
    """data/rulesheets/hexLG13.kif: place on an empty cell; white's swap on its first turn
    (canSwap kept only by white noops) mirrors black's stones through swapaxis; groups via a
    union-find over the adjacency relation; blackpath joins columns 1 and 13, whitepath rows a and
    m.  Roles black (0), white (1); base cell(r,c,p) = (r*13+(c-1))*2+p, control 338/339,
    canSwap 340; action 1+r*13+(c-1), swap 170."""
    N = 13

    def __init__(self):
        self.game = "hexLG13"
        self.role_count = 2
        self.num_bases = 2 * 169 + 3
        self.initial_state = (1 << 338) | (1 << 340)

    def base_name(self, i):
        if i == 338:
            return "(control black)"
        if i == 339:
            return "(control white)"
        if i == 340:
            return "canSwap"
        c, p = divmod(i, 2)
        return "(cell %s %d %s)" % ("abcdefghijklm"[c // 13], c % 13 + 1, "black" if p == 0 else "white")

    def action_count(self, role):
        return 170 if role == 0 else 171

    def legal_to_move(self, role, a):
        if a == 0:
            return "noop"
        if a == 170:
            return "swap"
        return "(place %s %d)" % ("abcdefghijklm"[(a - 1) // 13], (a - 1) % 13 + 1)

    def _owner(self, s, i):
        for p in (0, 1):
            if (s >> (2 * i + p)) & 1:
                return p
        return None

    def control(self, s):
        return 0 if (s >> 338) & 1 else 1

    def legal(self, s, role):
        if self.control(s) != role:
            return [0]
        out = [1 + i for i in range(169) if self._owner(s, i) is None]
        if role == 1 and (s >> 340) & 1:
            out.append(170)
        return out

    def _adjacent(self, j, k):
        # kif adjacent: same row +-1 col, same col +-1 row, (j-1, k+1), (j+1, k-1)
        for dj, dk in ((0, 1), (0, -1), (1, 0), (-1, 0), (-1, 1), (1, -1)):
            if 0 <= j + dj < 13 and 0 <= k + dk < 13:
                yield j + dj, k + dk

    def _path(self, s, p):
        parent = list(range(169))

        def find(a):
            while parent[a] != a:
                parent[a] = parent[parent[a]]
                a = parent[a]
            return a
        for i in range(169):
            if self._owner(s, i) != p:
                continue
            for j, k in self._adjacent(i // 13, i % 13):
                if self._owner(s, j * 13 + k) == p:
                    parent[find(i)] = find(j * 13 + k)
        if p == 0:
            a = {find(r * 13) for r in range(13) if self._owner(s, r * 13) == 0}
            b = {find(r * 13 + 12) for r in range(13) if self._owner(s, r * 13 + 12) == 0}
        else:
            a = {find(c) for c in range(13) if self._owner(s, c) == 1}
            b = {find(12 * 13 + c) for c in range(13) if self._owner(s, 12 * 13 + c) == 1}
        return bool(a & b)

    def is_terminal(self, s):
        return self._path(s, 0) or self._path(s, 1)

    def goal(self, s, role):
        return 100 if self._path(s, role) else 0

    def next_state(self, s, joint):
        mover = self.control(s)
        a = joint[mover]
        out = 0
        if a == 170:
            for i in range(169):
                if self._owner(s, i) == 0:          # swapaxis: (x, y) -> (letter y, number x)
                    r, c = divmod(i, 13)
                    out |= 1 << (2 * (c * 13 + r) + 1)
        else:
            for i in range(169):
                p = self._owner(s, i)
                if p is not None:
                    out |= 1 << (2 * i + p)
            if a:
                out |= 1 << (2 * (a - 1) + mover)
        out |= 1 << (338 + 1 - mover)
        if (s >> 340) & 1 and joint[1] == 0:
            out |= 1 << 340
        return out


class Amazons10(object):
    """data/rulesheets/amazons_10x10.kif: (turn p move) -> legalMove (move x1 y1 x2 y2) over
    openPath (recursive, one step at a time through unoccupied cells); (turn p fire) -> (fire x y)
    over openPath from justMoved; the other role noops; terminal when the role to play has no
    legalMove; goal 0 for the role to play, 100 for the other.  Roles white (0), black (1); base
    justMoved(x,y) = (x-1)*10+(y-1), cell(x,y,p) = 100+((x-1)*10+(y-1))*3+p, turn 400..403;
    actions noop, queen moves (x1, y1, dir n ne e se s sw w nw, distance), 2941+cell fire."""
    DIRS = [(0, 1), (1, 1), (1, 0), (1, -1), (0, -1), (-1, -1), (-1, 0), (-1, 1)]

    def __init__(self):
        self.game = "amazons_10x10"
        self.role_count = 2
        self.num_bases = 404
        self.moves = [None]
        for x in range(1, 11):
            for y in range(1, 11):
                for dx, dy in self.DIRS:
                    x2, y2 = x + dx, y + dy
                    while 1 <= x2 <= 10 and 1 <= y2 <= 10:
                        self.moves.append((x, y, x2, y2))
                        x2, y2 = x2 + dx, y2 + dy
        assert len(self.moves) == 2941
        self.move_index = {m: i for i, m in enumerate(self.moves) if m}
        s = 0
        for x, y in ((1, 4), (4, 1), (7, 1), (10, 4)):
            s |= 1 << self.cell(x, y, 0)
        for x, y in ((1, 7), (4, 10), (7, 10), (10, 7)):
            s |= 1 << self.cell(x, y, 1)
        self.initial_state = s | (1 << 400)

    def cell(self, x, y, p):
        return 100 + ((x - 1) * 10 + (y - 1)) * 3 + p

    def base_name(self, i):
        if i >= 400:
            return ["(turn white move)", "(turn white fire)", "(turn black move)", "(turn black fire)"][i - 400]
        if i < 100:
            return "(justMoved %d %d)" % (i // 10 + 1, i % 10 + 1)
        c, p = divmod(i - 100, 3)
        return "(cell %d %d %s)" % (c // 10 + 1, c % 10 + 1, ["white", "black", "arrow"][p])

    def action_count(self, role):
        return 3041

    def legal_to_move(self, role, a):
        if a == 0:
            return "noop"
        if a >= 2941:
            return "(fire %d %d)" % ((a - 2941) // 10 + 1, (a - 2941) % 10 + 1)
        return "(move %d %d %d %d)" % self.moves[a]

    def _occupied(self, s, x, y):
        return any((s >> self.cell(x, y, p)) & 1 for p in range(3))

    def _turn(self, s):
        for t in range(4):
            if (s >> (400 + t)) & 1:
                return t // 2, t % 2
        raise AssertionError("no turn base")

    def _open_path(self, s, x1, y1, d):
        dx, dy = d
        x2, y2 = x1 + dx, y1 + dy
        if not (1 <= x2 <= 10 and 1 <= y2 <= 10) or self._occupied(s, x2, y2):
            return []
        return [(x2, y2)] + self._open_path(s, x2, y2, d)

    def _legal_moves(self, s, role):
        player, phase = self._turn(s)
        out = []
        if player != role:
            return out
        if phase == 0:
            for x in range(1, 11):
                for y in range(1, 11):
                    if (s >> self.cell(x, y, role)) & 1:
                        for d in self.DIRS:
                            out += [self.move_index[(x, y, x2, y2)] for x2, y2 in self._open_path(s, x, y, d)]
        else:
            for i in range(100):
                if (s >> i) & 1:
                    for d in self.DIRS:
                        out += [2941 + (x2 - 1) * 10 + (y2 - 1)
                                for x2, y2 in self._open_path(s, i // 10 + 1, i % 10 + 1, d)]
        return sorted(out)

    def legal(self, s, role):
        if self._turn(s)[0] != role:
            return [0]
        return self._legal_moves(s, role)

    def is_terminal(self, s):
        return not self._legal_moves(s, self._turn(s)[0])

    def goal(self, s, role):
        return 0 if self._turn(s)[0] == role else 100

    def next_state(self, s, joint):
        player, phase = self._turn(s)
        a = joint[player]
        out = 0
        vacated = arrived = None
        if 0 < a < 2941:
            x1, y1, x2, y2 = self.moves[a]
            vacated, arrived = (x1, y1), (x2, y2)
            out |= 1 << self.cell(x2, y2, player)
            out |= 1 << ((x2 - 1) * 10 + (y2 - 1))
        elif a >= 2941:
            out |= 1 << (100 + (a - 2941) * 3 + 2)
        for x in range(1, 11):
            for y in range(1, 11):
                for p in range(3):
                    if (s >> self.cell(x, y, p)) & 1 and (x, y) != vacated:
                        out |= 1 << self.cell(x, y, p)
        nxt = (player, 1) if phase == 0 else (1 - player, 0)
        return out | (1 << (400 + 2 * nxt[0] + nxt[1]))


def make(game):
    if game == "breakthrough":
        return Breakthrough(8, "cellHolds", "breakthrough")
    if game == "breakthroughSmall":
        return Breakthrough(6, "cell", "breakthroughSmall")
    if game == "reversi":
        return Reversi()
    if game == "hexLG13":
        return HexLG13()
    if game == "amazons_10x10":
        return Amazons10()
    raise KeyError(game)


def state_to_words(s, num_bases):
    nw = (num_bases + 63) // 64
    return [(s >> (64 * i)) & ((1 << 64) - 1) for i in range(nw)]


def words_to_state(words):
    s = 0
    for i, w in enumerate(words):
        s |= int(w) << (64 * i)
    return s
