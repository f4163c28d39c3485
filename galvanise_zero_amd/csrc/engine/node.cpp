#include "node.h"

#include "tls.h"
#include "transformer.h"

#include <algorithm>
#include <cstdlib>
#include <limits>
#include <mutex>

#include <sys/mman.h>

namespace gz {

static_assert(sizeof(PuctNode) == 64, "node header must be one cache line");

static size_t node_bytes(int num_children, int role_count, int num_words) {
    size_t n = sizeof(PuctNode) + (sizeof(PuctNodeChild) + sizeof(PuctChildCold)) * num_children +
               sizeof(Score) * role_count;
    n = (n + 7) & ~size_t(7);
    n += sizeof(uint64_t) * num_words;
    return (n + 63) & ~size_t(63);   // aligned_alloc: size is a multiple of the alignment
}

// Node memory: nodes are variable-size (children count) and the tree churns through them (every
// expansion allocates one, every move releases the siblings' subtrees).  Nodes of up to 64 KiB are
// carved from 2 MiB chunks advised as transparent huge pages (a bench runner holds ~14 GB of trees:
// with 4 KiB pages nearly every cold node visit is also a TLB miss) and recycled per thread by
// 64-byte size class, without malloc's free lists (whose unlink checks touched cold neighbouring
// chunks: ~5 % of engine time).  A block freed on another thread joins that thread's lists; a
// thread's lists pass to a process-wide pool when it exits or destroys a pool (node_cache_flush),
// and new blocks come from that pool before a fresh chunk.  Chunks live as long as the process; larger nodes use aligned_alloc.
namespace {
constexpr size_t kNodeCacheClasses = 1024;     // blocks up to 64 KiB come from chunks
constexpr size_t kChunkBytes = size_t(2) << 20;

struct NodePool {   // process-wide: blocks of exited threads, per size class
    std::mutex mu;
    void* head[kNodeCacheClasses] = {};
};
NodePool& node_pool() {
    static NodePool* p = new NodePool();   // never destroyed (threads may exit during static teardown)
    return *p;
}

#if defined(__SANITIZE_ADDRESS__)
// AddressSanitizer builds (tests/test_transpositions.py) keep the recycling allocator: a block on a
// free list is poisoned whole (its link word too), so a use after free is caught even when the
// block is recycled; the list code unpoisons a link word only for the access itself.
#include <sanitizer/asan_interface.h>
inline void poison(void* p, size_t n) { ASAN_POISON_MEMORY_REGION(p, n); }
inline void unpoison(void* p, size_t n) { ASAN_UNPOISON_MEMORY_REGION(p, n); }
#else
inline void poison(void*, size_t) {}
inline void unpoison(void*, size_t) {}
#endif

inline void* link_of(void* p) {
    unpoison(p, sizeof(void*));
    void* n = *static_cast<void**>(p);
    poison(p, sizeof(void*));
    return n;
}
inline void set_link(void* p, void* n) {
    unpoison(p, sizeof(void*));
    *static_cast<void**>(p) = n;
    poison(p, sizeof(void*));
}

struct NodeCache {
    void* head[kNodeCacheClasses] = {};
    long blocks = 0;       // blocks on this thread's lists
    char* cur = nullptr;   // bump region of the current chunk
    char* end = nullptr;
    ~NodeCache() { flush(); }
    // hand every listed block to the process-wide pool
    void flush() {
        if (blocks == 0) return;
        NodePool& pool = node_pool();
        std::lock_guard<std::mutex> lk(pool.mu);
        for (size_t c = 0; c < kNodeCacheClasses; ++c) {
            void* p = head[c];
            if (p == nullptr) continue;
            void* last = p;
            for (void* n = link_of(last); n != nullptr; n = link_of(last)) last = n;
            set_link(last, pool.head[c]);
            pool.head[c] = p;
            head[c] = nullptr;
        }
        blocks = 0;
    }
    void* fresh(size_t bytes) {
        if (cur == nullptr || (size_t)(end - cur) < bytes) {
            void* chunk = std::aligned_alloc(kChunkBytes, kChunkBytes);
            if (chunk == nullptr) return nullptr;
            madvise(chunk, kChunkBytes, MADV_HUGEPAGE);   // advice only: 4 KiB pages if refused
            cur = static_cast<char*>(chunk);
            end = cur + kChunkBytes;
        }
        void* p = cur;
        cur += bytes;
        return p;
    }
};

void* node_alloc(size_t bytes) {   // bytes: a multiple of 64
    const size_t c = bytes / 64;
    if (c >= kNodeCacheClasses) return std::aligned_alloc(64, bytes);
    NodeCache& nc = tls_instance<NodeCache>();
    if (void* p = nc.head[c]) {
        nc.head[c] = link_of(p);
        nc.blocks--;
        unpoison(p, bytes);
        return p;
    }
    {   // blocks of exited threads / destroyed pools: take up to kRefill at once (one lock per
        // batch, not per node, when a new runner's threads draw on a destroyed one's trees)
        constexpr int kRefill = 64;
        NodePool& pool = node_pool();
        void* first = nullptr;
        {
            std::lock_guard<std::mutex> lk(pool.mu);
            first = pool.head[c];
            if (first != nullptr) {
                void* last = first;
                int k = 1;
                for (void* n = link_of(last); n != nullptr && k < kRefill; n = link_of(last), ++k) last = n;
                pool.head[c] = link_of(last);
                set_link(last, nullptr);
            }
        }
        if (first != nullptr) {
            void* rest = link_of(first);
            for (void* q = rest; q != nullptr; q = link_of(q)) nc.blocks++;
            nc.head[c] = rest;
            unpoison(first, bytes);
            return first;
        }
    }
    return nc.fresh(bytes);
}

void node_free(void* p, size_t bytes) {
    const size_t c = bytes / 64;
    if (c >= kNodeCacheClasses) {
        std::free(p);
        return;
    }
    NodeCache& nc = tls_instance<NodeCache>();
    poison(p, bytes);
    set_link(p, nc.head[c]);
    nc.head[c] = p;
    nc.blocks++;
}
}  // namespace

// A pool torn down on a thread that never runs its games (gz_runner_destroy on the caller's thread)
// frees every node onto that thread's lists: hand them to the process-wide pool, where the next
// runner's engine threads find them (instead of growing a second tree footprint).
void node_cache_flush() { tls_instance<NodeCache>().flush(); }

// node.cpp:111-149: children = cross product of every role's legal moves, role 0 outermost.
static inline void initChild(PuctNodeChild* child, PuctChildCold* cold, const JointMove& move) {
    child->to_node = nullptr;
    child->unselectable = false;
    child->m_flags = 0;
    child->m_score = 0.0f;
    child->m_visits = 0;
    child->m_inflight = 0;
    child->traversals = 0;
    child->policy_prob_orig = 1.0f;
    child->policy_prob = 1.0f;
    cold->use_minimax = false;
    cold->next_prob = 0.0f;
    cold->debug_node_score = 0.0f;
    cold->debug_puct_score = 0.0f;
    cold->move = move;
}

static int initialiseChildHelper(PuctNode* node, int role_index, int child_index, int role_count,
                                 const int* const* legals, const int* counts, JointMove* joint_move) {
    const bool final_role = role_index == role_count - 1;
    const int n = counts[role_index];
    const int* lg = legals[role_index];
    for (int ii = 0; ii < n; ++ii) {
        joint_move->set(role_index, lg[ii]);
        if (final_role) {
            initChild(node->getNodeChild(role_count, child_index), node->cold() + child_index, *joint_move);
            child_index++;
        } else {
            child_index = initialiseChildHelper(node, role_index + 1, child_index, role_count, legals, counts, joint_move);
        }
    }
    return child_index;
}

// node.cpp:42-109 + 153-221
PuctNode* PuctNode::create(const uint64_t* base_state, StateMachine* sm) {
    const int role_count = sm->roleCount();
    const int num_words = sm->numWords();
    sm->updateBases(base_state);

    int lead_role_index = 0;
    bool is_finalised = true;
    int total_children = 0;
    if (!sm->isTerminal()) {
        total_children = 1;
        is_finalised = false;
        int max_moves_for_a_role = 1;
        for (int ri = 0; ri < role_count; ++ri) {
            const int c = sm->legalCount(ri);
            total_children *= c;
            if (c > max_moves_for_a_role) {
                max_moves_for_a_role = c;
                lead_role_index = ri;
            }
        }
        if (max_moves_for_a_role > 1) {
            bool rest_one = true;
            for (int ri = 0; ri < role_count; ++ri)
                if (ri != lead_role_index && sm->legalCount(ri) > 1) rest_one = false;
            if (!rest_one) lead_role_index = PuctNode::lead_role_index_simultaneous;
        }
    }

    const size_t bytes = node_bytes(total_children, role_count, num_words);
    PuctNode* node = static_cast<PuctNode*>(node_alloc(bytes));
    node->parent = nullptr;
    node->in_parent = nullptr;
    node->visits = 0;
    node->inflight_visits = 0;
    node->ref_count = 1;
    node->unselectable_count = 0;
    node->num_children = (uint16_t)total_children;
    node->num_children_expanded = 0;
    node->puct_constant = 1.44f;
    node->is_finalised = is_finalised;
    node->force_terminal = false;
    node->dirichlet_noise_set = false;
    node->lead_role_index = (int16_t)lead_role_index;
    node->game_depth = 0;
    node->role_count = (uint8_t)role_count;
    node->num_words = (uint16_t)num_words;
    node->allocated_size = (uint32_t)bytes;
    for (int ii = 0; ii < role_count; ++ii) {
        node->setFinalScore(ii, 0.0f);
        node->setCurrentScore(ii, 0.0f);
    }
    std::copy(base_state, base_state + num_words, node->getBaseState());

    if (!node->is_finalised) {
        // the legal arrays once per role (not a virtual call per child)
        const int* legals[kMaxRoles];
        int counts[kMaxRoles];
        for (int ri = 0; ri < role_count; ++ri) {
            legals[ri] = sm->legalArray(ri);
            counts[ri] = sm->legalCount(ri);
        }
        JointMove move{};
        const int count = initialiseChildHelper(node, 0, 0, role_count, legals, counts, &move);
        (void)count;
    } else {
        for (int ii = 0; ii < role_count; ++ii) {
            const int score = sm->goalValue(ii);
            node->setFinalScore(ii, score / 100.0);
            node->setCurrentScore(ii, score / 100.0);
        }
    }
    return node;
}

void PuctNode::destroy(PuctNode* n) { node_free(n, n->allocated_size); }

void PuctNode::normaliseX() {
    float total_prediction = 0;
    for (int ii = 0; ii < num_children; ii++) total_prediction += children()[ii].policy_prob;
    if (total_prediction > std::numeric_limits<float>::min()) {
        for (int ii = 0; ii < num_children; ii++) children()[ii].policy_prob /= total_prediction;
    } else {
        for (int ii = 0; ii < num_children; ii++) children()[ii].policy_prob = 1.0 / num_children;
    }
}

// node.cpp:316-343: by to_node visits desc, ties by next_prob / policy_prob desc (std::sort)
Children PuctNode::sortedChildren(const PuctNode* node, bool next_probability) {
    Children children;
    children.reserve(node->num_children);
    for (int ii = 0; ii < node->num_children; ii++) children.push_back(node->getNodeChild(0, ii));
    auto f = [next_probability, node](const PuctNodeChild* a, const PuctNodeChild* b) {
        const int visits_a = a->to_node == nullptr ? 0 : a->to_node->visits;
        const int visits_b = b->to_node == nullptr ? 0 : b->to_node->visits;
        if (visits_a == visits_b) {
            if (next_probability) return node->coldOf(a).next_prob > node->coldOf(b).next_prob;
            return a->policy_prob > b->policy_prob;
        }
        return visits_a > visits_b;
    };
    std::sort(children.begin(), children.end(), f);
    return children;
}

// node.cpp:346-373: by traversals desc, ties by next_prob / policy_prob desc (std::sort)
Children PuctNode::sortedChildrenTraversals(const PuctNode* node, bool next_probability) {
    Children children;
    children.reserve(node->num_children);
    for (int ii = 0; ii < node->num_children; ii++) children.push_back(node->getNodeChild(0, ii));
    auto f = [next_probability, node](const PuctNodeChild* a, const PuctNodeChild* b) {
        const int traversals_a = a->traversals;
        const int traversals_b = b->traversals;
        if (traversals_a == traversals_b) {
            if (next_probability) return node->coldOf(a).next_prob > node->coldOf(b).next_prob;
            return a->policy_prob > b->policy_prob;
        }
        return traversals_a > traversals_b;
    };
    std::sort(children.begin(), children.end(), f);
    return children;
}

std::string PuctNode::moveString(const JointMove& move, const StateMachine* sm) {
    std::string res = "(";
    for (int ii = 0; ii < sm->roleCount(); ii++) {
        if (ii > 0) res += " ";
        res += sm->legalToMove(ii, move.get(ii));
    }
    return res + ")";
}

// node.cpp:449-461: planes of this node + its parent chain (num_prev_states of them)
void PuctNodeRequest::add(float* buf, const GdlBasesTransformer* transformer) const {
    std::vector<const uint64_t*> prev_states;
    const PuctNode* cur = node->parent;
    for (int ii = 0; ii < transformer->getNumberPrevStates(); ii++) {
        if (cur != nullptr) {
            prev_states.push_back(cur->getBaseState());
            cur = cur->parent;
        }
    }
    transformer->toChannels(node->getBaseState(), prev_states, buf);
}

// node.cpp:463-511
void PuctNodeRequest::reply(const ModelResult& result, const GdlBasesTransformer* transformer) {
    const int role_count = transformer->getNumberPolicies();
    float total_prediction = 0.0f;
    const float* raw_policy = result.getPolicy(node->lead_role_index);
    const PuctChildCold* cold = node->cold();
    for (int ii = 0; ii < node->num_children; ii++) {
        PuctNodeChild* c = node->getNodeChild(role_count, ii);
        c->policy_prob_orig = raw_policy[cold[ii].move.get(node->lead_role_index)];
        c->policy_prob_orig = std::max(0.001f, c->policy_prob_orig);
        total_prediction += c->policy_prob_orig;
    }
    for (int ii = 0; ii < node->num_children; ii++) {
        PuctNodeChild* c = node->getNodeChild(role_count, ii);
        c->policy_prob_orig /= total_prediction;
        c->policy_prob = c->policy_prob_orig;
    }
    for (int ri = 0; ri < role_count; ri++) {
        float s = result.getReward(ri);
        if (transformer->getNumberRewards() == 3) {
            const float mid = result.getReward(2) / 2.0f;
            s += mid;
        }
        if (s > 1.0) s = 1.0f;
        else if (s < 0.0) s = 0.0f;
        node->setFinalScore(ri, s);
        node->setCurrentScore(ri, node->getFinalScore(ri, true));
    }
}

}  // namespace gz
