// Native state machines restating the GDL rule sheets the BASELINE configs use.
//
// Breakthrough N x N  (data/rulesheets/breakthrough.kif, N=8, base term "cellHolds";
//                      data/rulesheets/breakthroughSmall.kif, N=6, base term "cell")
//   roles: white (moves +y), black (moves -y); white starts (init (control white)).
//   legal: forward onto an empty cell; diagonal onto any cell not holding an own piece; the
//          non-mover plays noop.  next: mover's piece moves (captures), control flips.
//   terminal/goal: whiteWin = a white piece on row N or no black piece; blackWin = a black piece
//          on row 1 or no white piece; winner 100, loser 0.
//
// Canonical base order (this build): cell(x,y,role) -> ((x-1)*N + (y-1))*2 + role, x,y in 1..N,
// role 0=white 1=black; then control(white) = 2N^2, control(black) = 2N^2+1.
// Canonical action order per role (1 + N(N-1) + 2(N-1)^2 = 155 for N=8, 81 for N=6):
//   0 noop | forward moves, x-major then y1 | right diagonals (x2=x1+1), y1-major then x1 |
//   left diagonals (x2=x1-1), y1-major then x1.
#include "sm.h"

#include <memory>

namespace gz {

namespace {

class Breakthrough : public StateMachine {
public:
    Breakthrough(int n, const char* game, const char* cell_term) : N(n), game(game), cell_term(cell_term) {
        nbases = 2 * N * N + 2;
        nwords = (nbases + 63) / 64;
        nactions = 1 + N * (N - 1) + 2 * (N - 1) * (N - 1);
        for (int role = 0; role < 2; ++role) {
            from_[role].assign(nactions, -1);
            to_[role].assign(nactions, -1);
            for (int x = 1; x <= N; ++x)
                for (int k = 0; k < N - 1; ++k) {
                    int y1 = role == 0 ? k + 1 : k + 2;
                    int y2 = role == 0 ? y1 + 1 : y1 - 1;
                    define(role, 1 + (x - 1) * (N - 1) + k, x, y1, x, y2);
                }
            for (int k = 0; k < N - 1; ++k)
                for (int j = 0; j < N - 1; ++j) {
                    int y1 = role == 0 ? k + 1 : k + 2;
                    int y2 = role == 0 ? y1 + 1 : y1 - 1;
                    define(role, 1 + N * (N - 1) + k * (N - 1) + j, j + 1, y1, j + 2, y2);
                    define(role, 1 + N * (N - 1) + (N - 1) * (N - 1) + k * (N - 1) + j, j + 2, y1, j + 1, y2);
                }
        }
        init.assign(nwords, 0);
        for (int x = 1; x <= N; ++x) {
            for (int y = 1; y <= 2; ++y) bs_set(init.data(), cellBase(x, y, 0), true);
            for (int y = N - 1; y <= N; ++y) bs_set(init.data(), cellBase(x, y, 1), true);
        }
        bs_set(init.data(), 2 * N * N + 0, true);
        row1 = 0;
        rowN = 0;
        for (int x = 1; x <= N; ++x) {
            row1 |= 1ull << bit(x, 1);
            rowN |= 1ull << bit(x, N);
        }
        // lookup tables instead of divisions by the run-time N: base -> bitboard bit, square -> x / y
        // and square -> base of each role
        base_bit.assign(2 * N * N, 0);
        for (int cell = 0; cell < N * N; ++cell) base_bit[2 * cell] = base_bit[2 * cell + 1] = (uint8_t)bit(cell / N + 1, cell % N + 1);
        sq_x.assign(N * N, 0);
        sq_y.assign(N * N, 0);
        for (int r = 0; r < 2; ++r) sq_base[r].assign(N * N, 0);
        for (int b = 0; b < N * N; ++b) {
            sq_x[b] = (uint8_t)(b % N + 1);
            sq_y[b] = (uint8_t)(b / N + 1);
            for (int r = 0; r < 2; ++r) sq_base[r][b] = (uint16_t)cellBase(b % N + 1, b / N + 1, r);
        }
        updateBases(init.data());
    }

    StateMachine* dupe() const override { return new Breakthrough(*this); }
    std::string name() const override { return game; }
    int roleCount() const override { return 2; }
    std::string roleName(int role) const override { return role == 0 ? "white" : "black"; }
    int numBases() const override { return nbases; }
    std::string baseName(int i) const override {
        if (i >= 2 * N * N) return std::string("(control ") + (i == 2 * N * N ? "white" : "black") + ")";
        int cell = i / 2, p = i % 2;
        int x = cell / N + 1, y = cell % N + 1;
        return "(" + cell_term + " " + std::to_string(x) + " " + std::to_string(y) + " " +
               (p == 0 ? "white" : "black") + ")";
    }
    int actionCount(int) const override { return nactions; }
    std::string legalToMove(int role, int a) const override {
        if (a == 0) return "noop";
        int f = from_[role][a], t = to_[role][a];
        return "(move " + std::to_string(f % N + 1) + " " + std::to_string(f / N + 1) + " " +
               std::to_string(t % N + 1) + " " + std::to_string(t / N + 1) + ")";
    }
    const uint64_t* initialState() const override { return init.data(); }

    void updateBases(const uint64_t* bs) override {
        pieces[0] = pieces[1] = 0;
        for (int w = 0; w < nwords; ++w) {
            uint64_t word = bs[w];
            while (word) {
                const int b = __builtin_ctzll(word) + 64 * w;
                word &= word - 1;
                if (b < 2 * N * N) pieces[b & 1] |= 1ull << base_bit[b];
            }
        }
        mover = bs_get(bs, 2 * N * N) ? 0 : 1;
        white_win = (pieces[0] & rowN) != 0 || pieces[1] == 0;
        black_win = (pieces[1] & row1) != 0 || pieces[0] == 0;
        terminal = white_win || black_win;
        // legals: mover gets its moves (ascending action index), other role noop
        legals[1 - mover].assign(1, 0);
        legals[mover].clear();
        uint64_t amap[4] = {0, 0, 0, 0};
        const uint64_t own = pieces[mover], opp = pieces[1 - mover];
        const int dy = mover == 0 ? 1 : -1;
        uint64_t m = own;
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            const int x = sq_x[b], y = sq_y[b], y2 = y + dy;
            if (y2 < 1 || y2 > N) continue;
            const uint64_t fwd = 1ull << bit(x, y2);
            if (!((own | opp) & fwd)) markAction(amap, fwdAction(mover, x, y));
            if (x < N && !(own & (1ull << bit(x + 1, y2)))) markAction(amap, diagAction(mover, x, y, +1));
            if (x > 1 && !(own & (1ull << bit(x - 1, y2)))) markAction(amap, diagAction(mover, x, y, -1));
        }
        for (int w = 0; w < 4; ++w) {
            uint64_t word = amap[w];
            while (word) {
                legals[mover].push_back(__builtin_ctzll(word) + 64 * w);
                word &= word - 1;
            }
        }
    }

    int legalCount(int role) const override { return (int)legals[role].size(); }
    int legal(int role, int i) const override { return legals[role][i]; }
    const int* legalArray(int role) const override { return legals[role].data(); }
    bool isTerminal() const override { return terminal; }
    int goalValue(int role) const override { return (role == 0 ? white_win : black_win) ? 100 : 0; }

    void nextState(const JointMove& move, uint64_t* out) override {
        uint64_t p[2] = {pieces[0], pieces[1]};
        int next_mover = mover;
        for (int role = 0; role < 2; ++role) {
            const int a = move.get(role);
            if (a == 0) continue;
            const uint64_t f = 1ull << from_[role][a], t = 1ull << to_[role][a];
            p[role] = (p[role] & ~f) | t;
            p[1 - role] &= ~t;
        }
        next_mover = 1 - mover;
        std::memset(out, 0, sizeof(uint64_t) * nwords);
        for (int role = 0; role < 2; ++role) {
            uint64_t m = p[role];
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                bs_set(out, sq_base[role][b], true);
            }
        }
        bs_set(out, 2 * N * N + next_mover, true);
    }

private:
    int bit(int x, int y) const { return (y - 1) * N + (x - 1); }
    int cellBase(int x, int y, int p) const { return ((x - 1) * N + (y - 1)) * 2 + p; }
    int fwdAction(int role, int x, int y1) const {
        return 1 + (x - 1) * (N - 1) + (role == 0 ? y1 - 1 : y1 - 2);
    }
    int diagAction(int role, int x1, int y1, int dx) const {
        const int k = role == 0 ? y1 - 1 : y1 - 2;
        if (dx > 0) return 1 + N * (N - 1) + k * (N - 1) + (x1 - 1);
        return 1 + N * (N - 1) + (N - 1) * (N - 1) + k * (N - 1) + (x1 - 2);
    }
    static void markAction(uint64_t* amap, int a) { amap[a >> 6] |= 1ull << (a & 63); }
    void define(int role, int a, int x1, int y1, int x2, int y2) {
        from_[role][a] = bit(x1, y1);
        to_[role][a] = bit(x2, y2);
    }

    int N;
    std::string game, cell_term;
    int nbases, nwords, nactions;
    std::vector<int> from_[2], to_[2];
    std::vector<uint64_t> init;
    uint64_t row1, rowN;
    std::vector<uint8_t> base_bit, sq_x, sq_y;
    std::vector<uint16_t> sq_base[2];

    // state of the last updateBases
    uint64_t pieces[2] = {0, 0};
    int mover = 0;
    bool white_win = false, black_win = false, terminal = false;
    std::vector<int> legals[2];
};

}  // namespace

StateMachine* create_more_state_machine(const std::string& name);   // games_more.cpp

StateMachine* create_state_machine(const std::string& name) {
    if (name == "breakthrough") return new Breakthrough(8, "breakthrough", "cellHolds");
    if (name == "breakthroughSmall") return new Breakthrough(6, "breakthroughSmall", "cell");
    if (name == "bt_7") return new Breakthrough(7, "bt_7", "cellHolds");
    return create_more_state_machine(name);
}

std::vector<std::string> known_games() {
    return {"breakthrough", "breakthroughSmall", "bt_7", "reversi", "hexLG13", "amazons_10x10"};
}

}  // namespace gz
