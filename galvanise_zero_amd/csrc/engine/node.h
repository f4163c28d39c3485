// PUCT tree node.  Restates PuctNode / PuctNodeChild (reference src/cpp/puct/node.h:42-215,
// node.cpp:42-221): one variable-size allocation per node holding the children (one per joint
// move in the cross product of the roles' legal moves), the per-role current / final scores and the
// node's base state.
#pragma once

#include "sm.h"

#include <cstdint>
#include <vector>

namespace gz {

typedef float Score;

struct PuctNode;
class GdlBasesTransformer;

struct PuctNodeChild {
    PuctNode* to_node;
    bool unselectable;
    bool use_minimax;
    uint32_t traversals;
    float policy_prob_orig;
    float policy_prob;
    float next_prob;
    Score debug_node_score;
    Score debug_puct_score;
    JointMove move;
};

typedef std::vector<const PuctNodeChild*> Children;

struct PuctNode {
    static constexpr int lead_role_index_simultaneous = -1;

    const PuctNode* parent;
    uint32_t visits;
    uint16_t inflight_visits;
    uint16_t ref_count;
    uint16_t unselectable_count;
    uint16_t num_children;
    uint16_t num_children_expanded;
    float puct_constant;
    bool is_finalised;
    bool force_terminal;
    bool dirichlet_noise_set;
    int16_t lead_role_index;
    uint16_t game_depth;
    uint8_t role_count;
    uint16_t num_words;
    uint32_t allocated_size;
    // Current scores live in the header: together with visits / is_finalised / unselectable_count
    // they are all a parent's selection passes read of a child node, and the header is one 64-byte
    // line (nodes are 64-byte aligned), so each child costs one cache line, not two.
    Score current[kMaxRoles];

    // trailing storage: children[num_children] | final[R] | basestate words
    PuctNodeChild* children() { return reinterpret_cast<PuctNodeChild*>(this + 1); }
    const PuctNodeChild* children() const { return reinterpret_cast<const PuctNodeChild*>(this + 1); }
    PuctNodeChild* getNodeChild(int, int i) { return children() + i; }
    const PuctNodeChild* getNodeChild(int, int i) const { return children() + i; }

    Score* scoresPtr() { return reinterpret_cast<Score*>(children() + num_children); }
    const Score* scoresPtr() const { return reinterpret_cast<const Score*>(children() + num_children); }

    Score getCurrentScore(int role) const { return current[role]; }
    void setCurrentScore(int role, Score s) { current[role] = s; }
    Score getFinalScore(int role, bool clamp = false) const {
        Score s = scoresPtr()[role];
        if (clamp) s = s < 0.0f ? 0.0f : (s > 1.0f ? 1.0f : s);
        return s;
    }
    void setFinalScore(int role, Score s) { scoresPtr()[role] = s; }

    uint64_t* getBaseState() { return reinterpret_cast<uint64_t*>(basestateOffset()); }
    const uint64_t* getBaseState() const { return reinterpret_cast<const uint64_t*>(basestateOffset()); }

    bool isTerminal() const { return force_terminal || num_children == 0; }

    // node.h:177-198 (normaliseX): renormalise policy_prob, uniform if everything vanished
    void normaliseX();

    static PuctNode* create(const uint64_t* base_state, StateMachine* sm);
    static void destroy(PuctNode* n);

    static Children sortedChildren(const PuctNode* node, bool next_probability = false);
    static Children sortedChildrenTraversals(const PuctNode* node, bool next_probability = false);

    static std::string moveString(const JointMove& move, const StateMachine* sm);

private:
    char* basestateOffset() const {
        uintptr_t p = reinterpret_cast<uintptr_t>(scoresPtr() + role_count);
        p = (p + 7) & ~uintptr_t(7);
        return reinterpret_cast<char*>(p);
    }
};

// Rows returned by the network for one request (scheduler.h:20-49 ModelResult).
struct ModelResult {
    const float* policies[kMaxRoles];
    float rewards[4];
    const float* getPolicy(int i) const { return policies[i]; }
    float getReward(int i) const { return rewards[i]; }
};

// node.h:222-241: the evaluation request of one new node.
class PuctNodeRequest {
public:
    explicit PuctNodeRequest(PuctNode* node) : node(node) {}
    const uint64_t* getBaseState() const { return node->getBaseState(); }
    void add(float* buf, const GdlBasesTransformer* transformer) const;
    void reply(const ModelResult& result, const GdlBasesTransformer* transformer);

private:
    PuctNode* node;
};

}  // namespace gz
