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

// A child entry is split in two records (build layout, not the reference's): the hot one holds
// exactly what a selection pass reads -- 32 bytes, two entries per cache line -- and the cold one
// (the joint move, the next-move probability, diagnostics) lives in a parallel array after the hot
// array (PuctNode::cold).  Selection streams the hot array only.
struct PuctNodeChild {
    PuctNode* to_node;
    uint32_t traversals;
    float policy_prob_orig;
    float policy_prob;
    // Mirror of the fields of to_node a selection pass over the parent reads: kept current by
    // PuctNode::syncParent() at every change of to_node, so the selection streams the parent's child
    // array instead of dereferencing one node per child.  Valid while to_node != nullptr.
    Score m_score;           // to_node's current score for the parent's lead role
    uint32_t m_visits;
    uint16_t m_inflight;
    bool unselectable;
    uint8_t m_flags;         // mirror: kMirrorFinalised | kMirrorAllUnselectable
};
static_assert(sizeof(PuctNodeChild) == 32, "hot child entry: 32 bytes");

struct PuctChildCold {
    JointMove move;
    float next_prob;
    Score debug_node_score;
    Score debug_puct_score;
    bool use_minimax;
};

constexpr uint8_t kMirrorFinalised = 1, kMirrorAllUnselectable = 2;

typedef std::vector<const PuctNodeChild*> Children;

struct PuctNode {
    static constexpr int lead_role_index_simultaneous = -1;

    const PuctNode* parent;
    PuctNodeChild* in_parent;   // the parent's child entry mirroring this node (null for a root)
    // Current scores live in the header: together with visits / is_finalised / unselectable_count
    // they are what the parent's mirror copies; the header is one 64-byte line (nodes are 64-byte
    // aligned).
    Score current[kMaxRoles];
    uint32_t visits;
    float puct_constant;
    uint32_t allocated_size;
    uint16_t inflight_visits;
    uint16_t ref_count;
    uint16_t unselectable_count;
    uint16_t num_children;
    uint16_t num_children_expanded;
    int16_t lead_role_index;
    uint16_t game_depth;
    uint16_t num_words;
    bool is_finalised;
    bool force_terminal;
    bool dirichlet_noise_set;
    uint8_t role_count;

    // refresh the parent's mirror entry after a change of visits / current / inflight_visits /
    // is_finalised / unselectable_count
    void syncParent() {
        PuctNodeChild* e = in_parent;
        if (e == nullptr) return;
        const int lead = parent->lead_role_index < 0 ? 0 : parent->lead_role_index;
        e->m_score = current[lead];
        e->m_visits = visits;
        e->m_inflight = inflight_visits;
        e->m_flags = (uint8_t)((is_finalised ? kMirrorFinalised : 0) |
                               (num_children > 0 && unselectable_count == num_children ? kMirrorAllUnselectable : 0));
    }

    // trailing storage: children[num_children] (hot) | cold[num_children] | final[R] | basestate words
    PuctNodeChild* children() { return reinterpret_cast<PuctNodeChild*>(this + 1); }
    const PuctNodeChild* children() const { return reinterpret_cast<const PuctNodeChild*>(this + 1); }
    PuctNodeChild* getNodeChild(int, int i) { return children() + i; }
    const PuctNodeChild* getNodeChild(int, int i) const { return children() + i; }
    PuctChildCold* cold() { return reinterpret_cast<PuctChildCold*>(children() + num_children); }
    const PuctChildCold* cold() const { return reinterpret_cast<const PuctChildCold*>(children() + num_children); }
    // the cold record of one of this node's child entries
    PuctChildCold& coldOf(const PuctNodeChild* c) { return cold()[c - children()]; }
    const PuctChildCold& coldOf(const PuctNodeChild* c) const { return cold()[c - children()]; }
    const JointMove& moveOf(const PuctNodeChild* c) const { return coldOf(c).move; }

    Score* scoresPtr() { return reinterpret_cast<Score*>(cold() + num_children); }
    const Score* scoresPtr() const { return reinterpret_cast<const Score*>(cold() + num_children); }

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
    const PuctNode* target() const { return node; }
    const uint64_t* getBaseState() const { return node->getBaseState(); }
    void add(float* buf, const GdlBasesTransformer* transformer) const;
    void reply(const ModelResult& result, const GdlBasesTransformer* transformer);

private:
    PuctNode* node;
};

// Hands the calling thread's recycled node blocks to the process-wide pool (node.cpp).
void node_cache_flush();

}  // namespace gz
