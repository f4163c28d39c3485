// Native game state machines: the build's stand-in for the ggplib propnet StateMachine the
// reference drives (external, not vendored; interface used at puct/node.cpp:153-221,
// puct/evaluator.cpp:216-239, supervisor.cpp:20-32, selfplaymanager.cpp:134-150).
//
// A state is a bit vector of GDL bases ("BaseState"), stored as uint64 words.  Base order and
// action order are this build's canonical orders (documented per game in games.cpp); ggplib's
// own orders come from its propnet build and are unpinned.  Action counts per role
// match the reference model files' policy sizes (81 / 155 ...).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace gz {

constexpr int kMaxRoles = 4;

inline bool bs_get(const uint64_t* w, int i) { return (w[i >> 6] >> (i & 63)) & 1ull; }
inline void bs_set(uint64_t* w, int i, bool v) {
    if (v) w[i >> 6] |= (1ull << (i & 63));
    else w[i >> 6] &= ~(1ull << (i & 63));
}

// One joint move: an action index per role (ggplib JointMove, IndexType entries).
struct JointMove {
    int16_t a[kMaxRoles];
    int get(int role) const { return a[role]; }
    void set(int role, int v) { a[role] = (int16_t)v; }
    bool equals(const JointMove& o, int roles) const {
        for (int r = 0; r < roles; ++r)
            if (a[r] != o.a[r]) return false;
        return true;
    }
};

class StateMachine {
public:
    virtual ~StateMachine() {}
    virtual StateMachine* dupe() const = 0;
    virtual std::string name() const = 0;

    virtual int roleCount() const = 0;
    virtual std::string roleName(int role) const = 0;
    virtual int numBases() const = 0;
    int numWords() const { return (numBases() + 63) / 64; }
    virtual std::string baseName(int index) const = 0;     // GDL term, e.g. "(cellHolds 1 2 white)"
    virtual int actionCount(int role) const = 0;          // = policy size of the role
    virtual std::string legalToMove(int role, int action) const = 0;

    virtual const uint64_t* initialState() const = 0;

    // ggplib-style stateful queries
    virtual void updateBases(const uint64_t* bs) = 0;
    virtual int legalCount(int role) const = 0;
    virtual int legal(int role, int i) const = 0;         // i-th legal action (ascending index)
    virtual const int* legalArray(int role) const = 0;    // the legalCount(role) legal actions
    virtual bool isTerminal() const = 0;
    virtual int goalValue(int role) const = 0;            // 0..100
    virtual void nextState(const JointMove& move, uint64_t* out) = 0;
};

// Factory by game name ("breakthrough", "breakthroughSmall", ...).  nullptr if unknown.
StateMachine* create_state_machine(const std::string& name);
std::vector<std::string> known_games();

}  // namespace gz
