// Native state machines for the BASELINE configs 3-5 games, restating their GDL rule sheets:
//
// reversi (8x8 Othello, data/rulesheets/reversi.kif; model data/reversi_8x8/models/*.json)
//   roles black, red; black starts.  The role in control places a disc that brackets a run of
//   opponent discs in at least one of 8 directions (playerCanMoveAt); every bracketed run flips
//   (affected / affectedCell).  A role in control with no such move plays noop (legal noop when
//   not playerCanMove); the other role always plays noop; control alternates every turn.
//   terminal: neither role can move.  goal: more discs 100, fewer 0, equal 50 both.
//   bases: cell(x,y,c) -> ((x-1)*8 + (y-1))*2 + c (c 0 black, 1 red); control black 128, red 129.
//   actions (65 per role): 0 noop, 1 + (x-1)*8 + (y-1) = (move x y).
//
// hexLG13 (data/rulesheets/hexLG13.kif; model data/hexLG13/models/*.json: policies 170 / 171)
//   roles black, white; black starts.  The role in control places on an empty cell; white may
//   instead swap while canSwap holds (only on its first turn: canSwap survives only white noops).
//   swap: each black stone (r, c) becomes a white stone at (letter c, number r) (swapaxis) and the
//   black stones leave the board.  Adjacency (adjacent): (r, c+-1), (r+-1, c), (r-1, c+1),
//   (r+1, c-1).  blackpath: a black group touching columns 1 and 13; whitepath: a white group
//   touching rows a and m.  The rule sheet tracks groups incrementally in connected/owner/step
//   bases; this build keeps only the stones and finds the groups by flood fill (same relation).
//   terminal: either path.  goal: path owner 100, other 0.
//   bases: cell(r,c,p) -> ((r)*13 + (c-1))*2 + p (r = row letter a..m as 0..12, p 0 black 1 white);
//   control black 338, white 339; canSwap 340.
//   actions: 0 noop, 1 + r*13 + (c-1) = (place r c); white also 170 = swap.
//
// amazons_10x10 (data/rulesheets/amazons_10x10.kif; model data/amazons_10x10/models/*.json:
//   policies 3041 = noop + 2940 queen-line moves + 100 fires)
//   roles white, black; white starts.  A turn is two plies: (turn p move): move one of p's queens
//   along an open line (queenMove / openPath: 8 directions, through empty cells); (turn p fire):
//   fire an arrow along an open line from the justMoved square.  The other role plays noop.
//   terminal: the role to play has no legal move.  goal: the role to play 0, the other 100.
//   bases: justMoved(x,y) -> (x-1)*10 + (y-1); cell(x,y,p) -> 100 + ((x-1)*10 + (y-1))*3 + p
//   (p 0 white, 1 black, 2 arrow); turn white move 400, white fire 401, black move 402,
//   black fire 403.
//   actions: 0 noop; queen moves enumerated x1, y1, direction (n ne e se s sw w nw), distance;
//   2941 + (x-1)*10 + (y-1) = (fire x y).
//
// Base and action orders are this build's (ggplib's propnet orders are unpinned); the
// per-role action counts equal the reference model files' policy sizes.  The oracle restatements
// are in oracle/games_ref.py.
#include "sm.h"

#include <algorithm>

namespace gz {

namespace {

// ---- reversi -------------------------------------------------------------------------------
class Reversi : public StateMachine {
public:
    static constexpr int N = 8, NB = 2 * N * N + 2;
    Reversi() {
        init.assign((NB + 63) / 64, 0);
        bs_set(init.data(), cellBase(4, 4, 0), true);
        bs_set(init.data(), cellBase(4, 5, 1), true);
        bs_set(init.data(), cellBase(5, 4, 1), true);
        bs_set(init.data(), cellBase(5, 5, 0), true);
        bs_set(init.data(), 2 * N * N, true);
        updateBases(init.data());
    }
    StateMachine* dupe() const override { return new Reversi(*this); }
    std::string name() const override { return "reversi"; }
    int roleCount() const override { return 2; }
    std::string roleName(int r) const override { return r == 0 ? "black" : "red"; }
    int numBases() const override { return NB; }
    std::string baseName(int i) const override {
        if (i >= 2 * N * N) return std::string("(control ") + (i == 2 * N * N ? "black" : "red") + ")";
        const int c = i / 2;
        return "(cell " + std::to_string(c / N + 1) + " " + std::to_string(c % N + 1) + " " +
               (i % 2 == 0 ? "black" : "red") + ")";
    }
    int actionCount(int) const override { return 1 + N * N; }
    std::string legalToMove(int, int a) const override {
        if (a == 0) return "noop";
        return "(move " + std::to_string((a - 1) / N + 1) + " " + std::to_string((a - 1) % N + 1) + ")";
    }
    const uint64_t* initialState() const override { return init.data(); }

    void updateBases(const uint64_t* bs) override {
        for (int i = 0; i < N * N; ++i) board[i] = bs_get(bs, 2 * i) ? 1 : bs_get(bs, 2 * i + 1) ? 2 : 0;
        mover = bs_get(bs, 2 * N * N) ? 0 : 1;
        std::vector<int> moves[2];
        for (int c = 0; c < 2; ++c)
            for (int i = 0; i < N * N; ++i)
                if (canMoveAt(c + 1, i)) moves[c].push_back(1 + i);
        terminal = moves[0].empty() && moves[1].empty();
        legals[1 - mover].assign(1, 0);
        legals[mover] = moves[mover].empty() ? std::vector<int>{0} : moves[mover];
        int cnt[3] = {0, 0, 0};
        for (int i = 0; i < N * N; ++i) cnt[board[i]]++;
        goals[0] = cnt[1] > cnt[2] ? 100 : cnt[1] < cnt[2] ? 0 : 50;
        goals[1] = 100 - goals[0];
    }
    int legalCount(int r) const override { return (int)legals[r].size(); }
    int legal(int r, int i) const override { return legals[r][i]; }
    const int* legalArray(int r) const override { return legals[r].data(); }
    bool isTerminal() const override { return terminal; }
    int goalValue(int r) const override { return goals[r]; }

    void nextState(const JointMove& move, uint64_t* out) override {
        int b[N * N];
        std::copy(board, board + N * N, b);
        const int a = move.get(mover);
        if (a != 0) {
            const int i = a - 1, me = mover + 1, opp = 2 - mover;
            const int x = i / N, y = i % N;
            for (int d = 0; d < 8; ++d) {
                int run = 0, cx = x + DX[d], cy = y + DY[d];
                while (in(cx, cy) && board[cx * N + cy] == opp) { ++run; cx += DX[d]; cy += DY[d]; }
                if (run > 0 && in(cx, cy) && board[cx * N + cy] == me)
                    for (int k = 1; k <= run; ++k) b[(x + k * DX[d]) * N + (y + k * DY[d])] = me;
            }
            b[i] = me;
        }
        std::memset(out, 0, sizeof(uint64_t) * numWords());
        for (int i = 0; i < N * N; ++i)
            if (b[i]) bs_set(out, 2 * i + (b[i] - 1), true);
        bs_set(out, 2 * N * N + (1 - mover), true);
    }

private:
    static constexpr int DX[8] = {0, 0, 1, -1, -1, 1, 1, -1};   // n s e w nw ne se sw
    static constexpr int DY[8] = {1, -1, 0, 0, 1, 1, -1, -1};
    static bool in(int x, int y) { return (unsigned)x < (unsigned)N && (unsigned)y < (unsigned)N; }
    static int cellBase(int x, int y, int c) { return ((x - 1) * N + (y - 1)) * 2 + c; }
    bool canMoveAt(int me, int i) const {
        if (board[i]) return false;
        const int opp = 3 - me, x = i / N, y = i % N;
        for (int d = 0; d < 8; ++d) {
            int run = 0, cx = x + DX[d], cy = y + DY[d];
            while (in(cx, cy) && board[cx * N + cy] == opp) { ++run; cx += DX[d]; cy += DY[d]; }
            if (run > 0 && in(cx, cy) && board[cx * N + cy] == me) return true;
        }
        return false;
    }
    std::vector<uint64_t> init;
    int board[N * N] = {};
    int mover = 0, goals[2] = {50, 50};
    bool terminal = false;
    std::vector<int> legals[2];
};
constexpr int Reversi::DX[8];
constexpr int Reversi::DY[8];

// ---- hex (LG 13x13, with swap) -------------------------------------------------------------
class Hex : public StateMachine {
public:
    static constexpr int N = 13, NC = N * N, CTRL = 2 * NC, SWAPB = 2 * NC + 2, NB = 2 * NC + 3;
    static constexpr int SWAP_ACTION = 1 + NC;
    Hex() {
        init.assign((NB + 63) / 64, 0);
        bs_set(init.data(), CTRL, true);
        bs_set(init.data(), SWAPB, true);
        updateBases(init.data());
    }
    StateMachine* dupe() const override { return new Hex(*this); }
    std::string name() const override { return "hexLG13"; }
    int roleCount() const override { return 2; }
    std::string roleName(int r) const override { return r == 0 ? "black" : "white"; }
    int numBases() const override { return NB; }
    std::string baseName(int i) const override {
        if (i == CTRL) return "(control black)";
        if (i == CTRL + 1) return "(control white)";
        if (i == SWAPB) return "canSwap";
        const int c = i / 2;
        return "(cell " + std::string(1, (char)('a' + c / N)) + " " + std::to_string(c % N + 1) + " " +
               (i % 2 == 0 ? "black" : "white") + ")";
    }
    int actionCount(int r) const override { return r == 0 ? 1 + NC : 2 + NC; }
    std::string legalToMove(int, int a) const override {
        if (a == 0) return "noop";
        if (a == SWAP_ACTION) return "swap";
        return "(place " + std::string(1, (char)('a' + (a - 1) / N)) + " " + std::to_string((a - 1) % N + 1) + ")";
    }
    const uint64_t* initialState() const override { return init.data(); }

    void updateBases(const uint64_t* bs) override {
        for (int i = 0; i < NC; ++i) board[i] = bs_get(bs, 2 * i) ? 1 : bs_get(bs, 2 * i + 1) ? 2 : 0;
        mover = bs_get(bs, CTRL) ? 0 : 1;
        can_swap = bs_get(bs, SWAPB);
        black_path = path(1);
        white_path = path(2);
        legals[1 - mover].assign(1, 0);
        legals[mover].clear();
        for (int i = 0; i < NC; ++i)
            if (!board[i]) legals[mover].push_back(1 + i);
        if (mover == 1 && can_swap) legals[1].push_back(SWAP_ACTION);
    }
    int legalCount(int r) const override { return (int)legals[r].size(); }
    int legal(int r, int i) const override { return legals[r][i]; }
    const int* legalArray(int r) const override { return legals[r].data(); }
    bool isTerminal() const override { return black_path || white_path; }
    int goalValue(int r) const override { return (r == 0 ? black_path : white_path) ? 100 : 0; }

    void nextState(const JointMove& move, uint64_t* out) override {
        int b[NC];
        std::copy(board, board + NC, b);
        const int a = move.get(mover);
        bool swapped = false;
        if (a == SWAP_ACTION) {
            swapped = true;
            std::fill(b, b + NC, 0);
            for (int i = 0; i < NC; ++i)   // no frame rule on swap: only the mirrored stones remain
                if (board[i] == 1) b[(i % N) * N + i / N] = 2;   // (r, c) -> (letter c, number r)
        } else if (a != 0) {
            b[a - 1] = mover + 1;
        }
        std::memset(out, 0, sizeof(uint64_t) * numWords());
        for (int i = 0; i < NC; ++i)
            if (b[i]) bs_set(out, 2 * i + (b[i] - 1), true);
        bs_set(out, CTRL + (1 - mover), true);
        // next canSwap: canSwap and white does noop
        if (can_swap && !swapped && move.get(1) == 0) bs_set(out, SWAPB, true);
    }

private:
    // a group of `who` touching both edges: black columns 1 / 13, white rows a / m
    bool path(int who) const {
        int stack[NC], sp = 0;
        bool seen[NC] = {};
        for (int k = 0; k < N; ++k) {
            const int i = who == 1 ? k * N : k;   // black: (row k, col 1); white: (row a, col k+1)
            if (board[i] == who && !seen[i]) { seen[i] = true; stack[sp++] = i; }
        }
        static constexpr int DR[6] = {0, 0, 1, -1, -1, 1}, DC[6] = {1, -1, 0, 0, 1, -1};
        while (sp) {
            const int i = stack[--sp], r = i / N, c = i % N;
            if ((who == 1 ? c : r) == N - 1) return true;
            for (int d = 0; d < 6; ++d) {
                const int rr = r + DR[d], cc = c + DC[d];
                if ((unsigned)rr >= (unsigned)N || (unsigned)cc >= (unsigned)N) continue;
                const int j = rr * N + cc;
                if (board[j] == who && !seen[j]) { seen[j] = true; stack[sp++] = j; }
            }
        }
        return false;
    }
    std::vector<uint64_t> init;
    int board[NC] = {};
    int mover = 0;
    bool can_swap = true, black_path = false, white_path = false;
    std::vector<int> legals[2];
};

// ---- amazons 10x10 ---------------------------------------------------------------------------
class Amazons : public StateMachine {
public:
    static constexpr int N = 10, NC = N * N, CELL0 = NC, TURN0 = NC + 3 * NC, NB = TURN0 + 4;
    static constexpr int FIRE0 = 2941, NA = 3041;
    Amazons() {
        qmove.assign(NC * NC, -1);
        from_.assign(NA, -1);
        to_.assign(NA, -1);
        int a = 1;
        for (int x = 0; x < N; ++x)
            for (int y = 0; y < N; ++y)
                for (int d = 0; d < 8; ++d)
                    for (int cx = x + DX[d], cy = y + DY[d]; in(cx, cy); cx += DX[d], cy += DY[d]) {
                        qmove[(x * N + y) * NC + cx * N + cy] = a;
                        from_[a] = x * N + y;
                        to_[a] = cx * N + cy;
                        ++a;
                    }
        init.assign((NB + 63) / 64, 0);
        const int wq[4][2] = {{1, 4}, {4, 1}, {7, 1}, {10, 4}}, bq[4][2] = {{1, 7}, {4, 10}, {7, 10}, {10, 7}};
        for (auto& q : wq) bs_set(init.data(), CELL0 + ((q[0] - 1) * N + q[1] - 1) * 3 + 0, true);
        for (auto& q : bq) bs_set(init.data(), CELL0 + ((q[0] - 1) * N + q[1] - 1) * 3 + 1, true);
        bs_set(init.data(), TURN0 + 0, true);
        updateBases(init.data());
    }
    StateMachine* dupe() const override { return new Amazons(*this); }
    std::string name() const override { return "amazons_10x10"; }
    int roleCount() const override { return 2; }
    std::string roleName(int r) const override { return r == 0 ? "white" : "black"; }
    int numBases() const override { return NB; }
    std::string baseName(int i) const override {
        static const char* piece[3] = {"white", "black", "arrow"};
        static const char* turn[4] = {"(turn white move)", "(turn white fire)", "(turn black move)", "(turn black fire)"};
        if (i >= TURN0) return turn[i - TURN0];
        if (i < CELL0) return "(justMoved " + std::to_string(i / N + 1) + " " + std::to_string(i % N + 1) + ")";
        const int c = (i - CELL0) / 3;
        return "(cell " + std::to_string(c / N + 1) + " " + std::to_string(c % N + 1) + " " + piece[(i - CELL0) % 3] + ")";
    }
    int actionCount(int) const override { return NA; }
    std::string legalToMove(int, int a) const override {
        if (a == 0) return "noop";
        if (a >= FIRE0) return "(fire " + std::to_string((a - FIRE0) / N + 1) + " " + std::to_string((a - FIRE0) % N + 1) + ")";
        const int f = from_[a], t = to_[a];
        return "(move " + std::to_string(f / N + 1) + " " + std::to_string(f % N + 1) + " " +
               std::to_string(t / N + 1) + " " + std::to_string(t % N + 1) + ")";
    }
    const uint64_t* initialState() const override { return init.data(); }

    void updateBases(const uint64_t* bs) override {
        just = -1;
        for (int i = 0; i < NC; ++i) {
            board[i] = bs_get(bs, CELL0 + 3 * i) ? 1 : bs_get(bs, CELL0 + 3 * i + 1) ? 2 : bs_get(bs, CELL0 + 3 * i + 2) ? 3 : 0;
            if (bs_get(bs, i)) just = i;
        }
        phase = 0;
        for (int t = 0; t < 4; ++t)
            if (bs_get(bs, TURN0 + t)) phase = t;
        mover = phase >> 1;
        legals[1 - mover].assign(1, 0);
        std::vector<int>& L = legals[mover];
        L.clear();
        if ((phase & 1) == 0) {
            for (int i = 0; i < NC; ++i)
                if (board[i] == mover + 1) slide(i, [&](int j) { L.push_back(qmove[i * NC + j]); });
            std::sort(L.begin(), L.end());
        } else if (just >= 0) {
            slide(just, [&](int j) { L.push_back(FIRE0 + j); });
            std::sort(L.begin(), L.end());
        }
    }
    int legalCount(int r) const override { return (int)legals[r].size(); }
    int legal(int r, int i) const override { return legals[r][i]; }
    const int* legalArray(int r) const override { return legals[r].data(); }
    bool isTerminal() const override { return legals[mover].empty(); }
    int goalValue(int r) const override { return r == mover ? 0 : 100; }

    void nextState(const JointMove& move, uint64_t* out) override {
        int b[NC];
        std::copy(board, board + NC, b);
        const int a = move.get(mover);
        int nj = -1, nphase = phase;
        if (a >= FIRE0) {
            b[a - FIRE0] = 3;
            nphase = ((1 - mover) << 1);
        } else if (a > 0) {
            b[to_[a]] = b[from_[a]];
            b[from_[a]] = 0;
            nj = to_[a];
            nphase = (mover << 1) | 1;
        }
        std::memset(out, 0, sizeof(uint64_t) * numWords());
        for (int i = 0; i < NC; ++i)
            if (b[i]) bs_set(out, CELL0 + 3 * i + (b[i] - 1), true);
        if (nj >= 0) bs_set(out, nj, true);
        bs_set(out, TURN0 + nphase, true);
    }

private:
    static constexpr int DX[8] = {0, 1, 1, 1, 0, -1, -1, -1};   // n ne e se s sw w nw
    static constexpr int DY[8] = {1, 1, 0, -1, -1, -1, 0, 1};
    static bool in(int x, int y) { return (unsigned)x < (unsigned)N && (unsigned)y < (unsigned)N; }
    template <typename Fn>
    void slide(int i, Fn fn) const {
        const int x = i / N, y = i % N;
        for (int d = 0; d < 8; ++d)
            for (int cx = x + DX[d], cy = y + DY[d]; in(cx, cy) && !board[cx * N + cy]; cx += DX[d], cy += DY[d])
                fn(cx * N + cy);
    }
    std::vector<uint64_t> init;
    std::vector<int16_t> qmove;        // [from][to] -> action (-1: not on a queen line)
    std::vector<int> from_, to_;
    int board[NC] = {};
    int just = -1, phase = 0, mover = 0;
    std::vector<int> legals[2];
};
constexpr int Amazons::DX[8];
constexpr int Amazons::DY[8];

}  // namespace

StateMachine* create_more_state_machine(const std::string& name) {
    if (name == "reversi" || name == "reversi_8x8") return new Reversi();
    if (name == "hexLG13") return new Hex();
    if (name == "amazons_10x10") return new Amazons();
    return nullptr;
}

}  // namespace gz
