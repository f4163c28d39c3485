// PUCT evaluator: restates PuctEvaluator (reference src/cpp/puct/evaluator.h:31-160,
// evaluator.cpp:37-1510).  One instance per game; it owns the game tree and asks its scheduler for
// a network evaluation of every new non-trivial node (the coroutine parks inside evaluate()).
#pragma once

#include "config.h"
#include "node.h"
#include "rng.h"
#include "scheduler.h"

#include <unordered_map>
#include <vector>

namespace gz {

struct PathElement {
    PathElement(PuctNode* node, PuctNodeChild* choice, PuctNodeChild* best)
        : node(node), choice(choice), best(best) {}
    PuctNode* node;
    PuctNodeChild* choice;
    PuctNodeChild* best;
};
using Path = std::vector<PathElement>;

struct PuctNodeDebug {
    float score = 0;
    int lead_role_index = 0;
    int move_index = 0;
    std::vector<std::pair<int, int>> variation;
};

class PuctEvaluator {
public:
    PuctEvaluator(StateMachine* sm, NetworkScheduler* scheduler, const GdlBasesTransformer* transformer);
    ~PuctEvaluator();

    void updateConf(const PuctConfig* conf);
    void seed(uint64_t s) { rng.seed(s); }

    void setDirichletNoise(PuctNode* node);
    float priorScore(PuctNode* node, int depth) const;
    void setPuctConstant(PuctNode* node, int depth) const;
    float getTemperature(int depth) const;

    const PuctNodeChild* choose(const PuctNode* node);
    bool converged(int count) const;

    PuctNode* expandChild(PuctNode* parent, PuctNodeChild* child);
    void balanceFirstMoves(int max_moves);

    void reset(int game_depth);
    PuctNode* fastApplyMove(const PuctNodeChild* next);
    PuctNode* establishRoot(const uint64_t* current_state);
    void resetRootNode();
    const PuctNodeChild* onNextMove(int max_evaluations, double end_time = -1);
    void applyMove(const JointMove* move);

    const PuctNodeChild* chooseTopVisits(const PuctNode* node) const;
    const PuctNodeChild* chooseTemperature(const PuctNode* node);
    Children getProbabilities(PuctNode* node, float temperature, bool use_policy = true);

    int nodeCount() const { return number_of_nodes; }
    StateMachine* getSM() const { return sm; }
    const PuctNode* getRootNode() const { return root; }
    PuctNode* getRootNodeMutable() { return root; }

    void nodeDebug(int child_index, int max_variation_depth, PuctNodeDebug& info) const;

    // per onNextMove statistics (evaluator.h:101-125)
    struct PlayoutStats {
        void reset() { *this = PlayoutStats(); }
        int num_blocked = 0;
        int num_tree_playouts = 0;
        int num_evaluations = 0;
        int num_transpositions_attached = 0;
        int playouts_total_depth = 0;
        int playouts_max_depth = 0;
        int playouts_finals = 0;
    };
    const PlayoutStats& getStats() const { return stats; }
    long totalEvaluations() const { return total_evaluations; }
    long totalTreePlayouts() const { return total_tree_playouts; }
    long totalTranspositions() const { return total_transpositions; }
    long totalSpinEpochs() const { return total_spin_epochs; }

private:
    void removeNode(PuctNode*);
    void releaseNodes(PuctNode*);
    PuctNode* lookupNode(const uint64_t* bs, int depth);
    PuctNode* createNode(PuctNode* parent, const uint64_t* state);
    PuctNodeChild* selectChild(PuctNode* node, Path& path);
    PuctNodeChild* selectChildLiteral(PuctNode* node, int depth, float prior_score, double sqrt_node_visits,
                                      PuctNodeChild** best_out);
    bool chooseTopVisitsFast(const PuctNode* node, const PuctNodeChild** out) const;
    const PuctNodeChild* chooseTopVisitsExact(const PuctNode* node) const;
    bool convergedFast(int count, bool* out) const;
    bool convergedExact(int count) const;
    void backup(float* new_scores, const Path& path);
    int treePlayout(PuctNode* current, Path& path);
    void playoutWorker(int worker_id);
    void playoutMain(int max_evaluations, double end_time);

    // Root spin fast path (evaluator.cpp, "spin"): playouts that go root -> finalised winning
    // child, run without the full selection pass while provably nothing else can be chosen.
    struct SpinEpoch {
        static constexpr int kMaxWins = 8, kMaxWatched = 6, kMaxVisited = 96;
        enum : uint8_t { kWin = 0, kScored = 1, kPrior = 2 };
        const PuctNode* root = nullptr;
        uint32_t v_end = 0;          // the epoch holds while root->visits < v_end
        uint32_t retry_at = 0;       // after a failed build: next attempt at this root visit count
        int reach = 0;               // selection candidates (root-latch RNG draws per playout)
        int ncand = 0;               // wins + watched candidates, in sortedChildrenSelect order
        uint16_t cand[kMaxWins + kMaxWatched];
        uint8_t cand_kind[kMaxWins + kMaxWatched];
        uint16_t cand_pos[kMaxWins + kMaxWatched];   // position among the reached children (latch draw)
        uint16_t watched_flag[kMaxWatched];
        int nvisited = 0;            // children with visits > 0, in child order (FPU policy sum)
        uint16_t visited[kMaxVisited];
        bool watch_prior = false;    // an unexpanded child is watched: the exact FPU prior is needed
        float win_score = 0.f;
        double unwatched_bound = 0;  // upper bound of every unwatched candidate's score until v_end
        bool conv_false = false;     // converged() proved false for the epoch
        bool valid = false;
        bool fail_next = false;      // spinRun: the next playout fails the fast path (seen in the last run)
        bool regs_ok = false;        // spinRunRegs applies: no watched prior, every win a childless leaf
        double drift = 1.0;          // product of the policy rescalings (normaliseX) since the build
    };
    bool spinBuild();
    int spinRun(int limit, bool multi);
    int spinRunSlow(int limit, bool verify);
    int spinRunRegs(int limit);
    struct SpinSnapshot {
        std::vector<char> bytes;
        bool valid = false, fail_next = false;
        uint32_t v_end = 0;
        double drift = 1.0;
        Rng rng;
        int playouts_finals = 0, num_tree_playouts = 0;
        long total_tree_playouts = 0;
        bool operator==(const SpinSnapshot& o) const;
    };
    SpinSnapshot spinSnapshot() const;
    void spinRestore(const SpinSnapshot& s);
    SpinEpoch spin;
    Path spin_path;

    // Forced replies among tied finalised wins (selectChild): the reference returns the first of
    // them in sortedChildrenSelect order, which std::sort's permutation of all the node's keys
    // decides.  While every visit to the node since goes through that child, no other child is
    // touched (single-parent trees: mirror_ok), every key is unchanged, and so is the answer: an
    // entry holds (node, its visits and the child's traversals then) and is valid exactly while
    // the node's visits and the child's traversals grew alike.  Entries of freed nodes are cleared.
    struct ForcedEntry {
        const PuctNode* node = nullptr;
        uint32_t visits = 0, trav = 0;
        uint16_t child = 0, nch = 0;
    };
    static constexpr int kForcedSlots = 64;
    ForcedEntry forced_cache[kForcedSlots];
    static int forcedSlot(const PuctNode* n) { return (int)((reinterpret_cast<uintptr_t>(n) >> 6) % kForcedSlots); }

    struct MaskedKey {
        std::vector<uint64_t> w;
        bool operator==(const MaskedKey& o) const { return w == o.w; }
    };
    struct MaskedHash {
        size_t operator()(const MaskedKey& k) const;
    };
    MaskedKey maskedKey(const uint64_t* bs) const;

    const PuctConfig* conf = nullptr;
    StateMachine* sm;
    std::vector<uint64_t> basestate_expand_node;
    NetworkScheduler* scheduler;
    std::vector<uint64_t> hash_mask;

    int game_depth = 0;
    PuctNode* initial_root = nullptr;
    PuctNode* root = nullptr;

    std::unordered_map<MaskedKey, PuctNode*, MaskedHash> lookup;
    std::vector<PuctNode*> garbage;

    int number_of_nodes = 0;
    long node_allocated_memory = 0;
    long total_evaluations = 0;
    long total_tree_playouts = 0;   // diagnostics: NN-free playouts = tree playouts - evaluations
    long total_transpositions = 0;  // diagnostics: edges attached to an existing node (lookup_transpositions)
    long total_spin_epochs = 0;     // diagnostics: root spin epochs built (spinBuild)
    bool do_playouts = false;
    bool mirror_ok = true;   // every node has one parent: the child mirrors (node.h) are exact
    PlayoutStats stats;
    Rng rng;
};

double get_time();

// GZ_VERIFY_FASTPATH at run time (process-wide; gz_engine_set_verify_fastpath)
void set_verify_fastpath(bool on);
bool get_verify_fastpath();
long verified_decisions();

}  // namespace gz
