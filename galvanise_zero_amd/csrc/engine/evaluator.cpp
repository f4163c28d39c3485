// Restatement of src/cpp/puct/evaluator.cpp.  Float/double mixing follows the reference
// expression by expression (e.g. selectChild's double `score` against float `best_score`), and the
// library is compiled with -ffp-contract=off so every operation rounds as written (the reference's
// contraction behaviour depends on its unknown k273 build flags and is unpinned).
#include "evaluator.h"

#include "tls.h"
#include "transformer.h"

#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <limits>
#include <mutex>
#include <random>

namespace gz {

// log((1 + visits + 19652) / 19652) in float, as the reference computes it (evaluator.cpp:1300-1307):
// every selection at every node evaluates it (a root spin run once per playout, at consecutive
// visit counts), so the values for visits < 2^26 are tabulated, 64K at a time on first use, with
// the same expression and the same libm call (identical bits); larger counts call logf directly.
static float puct_log_direct(uint32_t visits) {
    const float cpuct_base_id = 19652.0f;
    return std::log((1 + visits + cpuct_base_id) / cpuct_base_id);
}

// Beyond the tables (visits >= 2^26: roots deep in an NN-free spin) the float argument of the log
// changes only every 8+ visits (float(1 + visits) has that granularity): a small direct-mapped
// cache of (argument, log) pairs, each one 64-bit word (a racing store is a whole pair), keyed by
// the argument's bits -- the same libm call on the same argument, far fewer of them.
static inline float puct_log_arg(uint32_t visits) {
    const float cpuct_base_id = 19652.0f;
    return (1 + visits + cpuct_base_id) / cpuct_base_id;
}
namespace {
std::atomic<uint64_t> g_large_log[1024];
}
static float puct_log_large(uint32_t visits) {
    const float arg = puct_log_arg(visits);
    const uint32_t a = __builtin_bit_cast(uint32_t, arg);
    std::atomic<uint64_t>& e = g_large_log[(a >> 3) & 1023];
    const uint64_t w = e.load(std::memory_order_relaxed);
    if ((uint32_t)(w >> 32) == a && w != 0) return __builtin_bit_cast(float, (uint32_t)w);
    const float v = std::log(arg);
    e.store((uint64_t)a << 32 | __builtin_bit_cast(uint32_t, v), std::memory_order_relaxed);
    return v;
}

namespace {
constexpr int kPuctLogBlockBits = 16, kPuctLogBlocks = 1024;   // visits < 2^26
std::atomic<float*> g_puct_log[kPuctLogBlocks];
std::mutex g_puct_log_mu;

__attribute__((noinline)) float* puct_log_block(uint32_t b) {
    std::lock_guard<std::mutex> lk(g_puct_log_mu);
    float* t = g_puct_log[b].load(std::memory_order_acquire);
    if (t == nullptr) {
        t = new float[1u << kPuctLogBlockBits];
        const uint32_t v0 = b << kPuctLogBlockBits;
        for (uint32_t i = 0; i < (1u << kPuctLogBlockBits); ++i) t[i] = puct_log_direct(v0 + i);
        g_puct_log[b].store(t, std::memory_order_release);
    }
    return t;
}
}  // namespace

static inline float puct_log(uint32_t visits) {
    const uint32_t b = visits >> kPuctLogBlockBits;
    if (b >= (uint32_t)kPuctLogBlocks) return puct_log_large(visits);
    float* t = g_puct_log[b].load(std::memory_order_acquire);
    if (__builtin_expect(t == nullptr, 0)) t = puct_log_block(b);
    return t[visits & ((1u << kPuctLogBlockBits) - 1)];
}

// puct_log at consecutive visit counts (a spin run): the current 64K block held, refreshed at its end;
// beyond the tables the last argument and its log
struct PuctLogCursor {
    const float* t = nullptr;
    uint32_t b = ~0u;
    float last_arg = -1.f, last_val = 0.f;
    inline float at(uint32_t visits) {
        const uint32_t vb = visits >> kPuctLogBlockBits;
        if (__builtin_expect(vb != b, 0)) {
            if (vb >= (uint32_t)kPuctLogBlocks) {
                const float arg = puct_log_arg(visits);
                if (arg != last_arg) {
                    last_arg = arg;
                    last_val = puct_log_large(visits);
                }
                return last_val;
            }
            t = g_puct_log[vb].load(std::memory_order_acquire);
            if (t == nullptr) t = puct_log_block(vb);
            b = vb;
        }
        return t[visits & ((1u << kPuctLogBlockBits) - 1)];
    }
};

// sqrt of a positive double as the one sqrtsd instruction (std::sqrt adds a domain check for errno;
// the result is the same correctly rounded value)
static inline double sqrt_pos(double x) { return _mm_cvtsd_f64(_mm_sqrt_sd(_mm_setzero_pd(), _mm_set_sd(x))); }


// GZ_SPIN_STATS=1: spin fast-path counters (process totals, printed at exit; diagnostics only)
namespace {
enum SpinStat {
    kSdBuilds, kSdBuildOk, kSdFailRoot, kSdFailUnselectable, kSdFailVisited, kSdFailInflight, kSdFailWinNode,
    kSdFailWinScore, kSdFailLatch, kSdFailFewWins, kSdFailOrder, kSdFailWatched, kSdRegsPlayouts,
    kSdSlowPlayouts, kSdOrdinaryPlayouts, kSdRetryWait, kSdSelect, kSdSelectSorted,
    // NN-free ordinary playouts by the root's finalised wins (0 / 1 / >= 2) and by where they end
    kSdFree0, kSdFree1, kSdFree2, kSdFreeD2, kSdFreeD3, kSdFreeD4, kSdFreeD5, kSdFreeD6, kSdFreeConv,
    kSdFreeX1Win,
    // playoutMain's exits, and the NN-free playouts of moves ending at each
    kSdExitFinal, kSdExitConvPlayouts, kSdExitConvEvals, kSdExitNonConvEvals, kSdExitOther,
    kSdFreeAtConvPlayouts, kSdFreeAtConvEvals, kSdFreeAtNonConvEvals,
    // register runs: how they end
    kSdRegRuns, kSdRegFailNoise, kSdRegFailLatch, kSdRegFailSep, kSdRegExpired,
    kSdLatchDraws,   // fast-path playouts that read a root-latch draw
    kSdCycSpin, kSdCycFree, kSdCycEval,   // TSC cycles in spin runs / NN-free / evaluating ordinary playouts
    kSdFreeLine,     // NN-free ordinary playouts whose path below the root is forced (1 child / forced win)
    kSdSelectForced, // selections decided by the forced-reply pass
    kSdCount
};
struct SpinStats {
    const bool on = std::getenv("GZ_SPIN_STATS") != nullptr;
    std::atomic<long> c[kSdCount] = {};
    ~SpinStats() {
        if (!on) return;
        static const char* names[kSdCount] = {
            "builds", "build_ok", "fail_root", "fail_unselectable", "fail_visited", "fail_inflight",
            "fail_win_node", "fail_win_score", "fail_latch", "fail_few_wins", "fail_order", "fail_watched",
            "regs_playouts", "slow_playouts", "ordinary_playouts", "retry_wait", "select", "select_sorted",
            "free_w0", "free_w1", "free_w2", "free_d2", "free_d3", "free_d4", "free_d5", "free_d6+", "free_converged",
            "free_d3_forced_win",
            "exit_finalised", "exit_conv_playouts", "exit_conv_evals", "exit_nonconv_evals", "exit_other",
            "free_at_conv_playouts", "free_at_conv_evals", "free_at_nonconv_evals",
            "reg_runs", "reg_fail_noise", "reg_fail_latch", "reg_fail_sep", "reg_expired", "latch_draws",
            "cyc_spin", "cyc_free", "cyc_eval", "free_line", "select_forced"};
        std::fprintf(stderr, "gz spin stats:");
        for (int i = 0; i < kSdCount; ++i) std::fprintf(stderr, " %s=%ld", names[i], c[i].load());
        std::fprintf(stderr, "\n");
    }
};
SpinStats g_spin_stats;
// per-thread counts, added to the process totals when the thread exits (16 engine threads adding
// to shared atomics per selection took 30 % of a profiled run's samples)
struct SpinStatsLocal {
    long c[kSdCount] = {};
    ~SpinStatsLocal() {
        for (int i = 0; i < kSdCount; ++i)
            if (c[i]) g_spin_stats.c[i].fetch_add(c[i], std::memory_order_relaxed);
    }
};
inline void sd(SpinStat i, long n) {
    if (__builtin_expect(g_spin_stats.on, 0)) tls_instance<SpinStatsLocal>().c[i] += n;
}
inline int spin_dump_at() {
    static const int v = [] {
        const char* e = std::getenv("GZ_SPIN_DUMP");
        return e != nullptr ? std::atoi(e) : -1;
    }();
    return v;
}
inline void sd(SpinStat i, long n = 1);
}  // namespace

#define GZ_ASSERT(cond)                                                                     \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "gz assertion failed: %s (%s:%d)\n", #cond, __FILE__, __LINE__); \
            std::abort();                                                                   \
        }                                                                                   \
    } while (0)

double get_time() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

size_t PuctEvaluator::MaskedHash::operator()(const MaskedKey& k) const {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint64_t w : k.w) {
        h ^= w + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    }
    return (size_t)h;
}

PuctEvaluator::MaskedKey PuctEvaluator::maskedKey(const uint64_t* bs) const {
    MaskedKey k;
    k.w.resize(hash_mask.size());
    for (size_t i = 0; i < hash_mask.size(); ++i) k.w[i] = bs[i] & hash_mask[i];
    return k;
}

PuctEvaluator::PuctEvaluator(StateMachine* sm, NetworkScheduler* scheduler, const GdlBasesTransformer* transformer)
    : sm(sm), scheduler(scheduler) {
    basestate_expand_node.assign(sm->numWords(), 0);
    hash_mask = transformer->createHashMask(sm->numBases());
}

PuctEvaluator::~PuctEvaluator() { reset(0); }

void PuctEvaluator::updateConf(const PuctConfig* c) { conf = c; }

// evaluator.cpp:102-140
void PuctEvaluator::removeNode(PuctNode* node) {
    if (conf->lookup_transpositions) lookup.erase(maskedKey(node->getBaseState()));
    ForcedEntry& fe = forced_cache[forcedSlot(node)];
    if (fe.node == node) fe.node = nullptr;
    node_allocated_memory -= node->allocated_size;
    PuctNode::destroy(node);
    number_of_nodes--;
}

// A transposed node (lookup_transpositions) is referenced by several parents, but its mirror entry
// (in_parent) and its parent pointer name the first one only.  When that edge is dropped and the
// node survives through another parent, both are cleared: syncParent() would otherwise write into
// the freed parent's child array, and createSample / the planes' previous state would read the
// freed parent (the reference reads it there: evaluator.cpp:102-140 never updates `parent`).
static inline void detachEdge(PuctNodeChild* edge, PuctNode* node) {
    if (node->ref_count > 0 && node->in_parent == edge) {
        node->in_parent = nullptr;
        node->parent = nullptr;
    }
}

void PuctEvaluator::releaseNodes(PuctNode* current) {
    const int role_count = sm->roleCount();
    for (int ii = 0; ii < current->num_children; ii++) {
        PuctNodeChild* child = current->getNodeChild(role_count, ii);
        if (child->to_node != nullptr) {
            PuctNode* next_node = child->to_node;
            if (next_node->ref_count <= 0) continue;   // cycle guard
            child->to_node = nullptr;
            next_node->ref_count--;
            if (next_node->ref_count == 0) {
                releaseNodes(next_node);
                garbage.push_back(next_node);
            } else {
                detachEdge(child, next_node);
            }
        }
    }
}

// evaluator.cpp:144-163
PuctNode* PuctEvaluator::lookupNode(const uint64_t* bs, int depth) {
    if (!conf->lookup_transpositions) return nullptr;
    auto found = lookup.find(maskedKey(bs));
    if (found != lookup.end()) {
        PuctNode* result = found->second;
        if (result->game_depth != depth) return nullptr;
        return result;
    }
    return nullptr;
}

// evaluator.cpp:165-214
PuctNode* PuctEvaluator::createNode(PuctNode* parent, const uint64_t* state) {
    PuctNode* new_node = PuctNode::create(state, sm);
    if (conf->lookup_transpositions) lookup.emplace(maskedKey(new_node->getBaseState()), new_node);
    number_of_nodes++;
    node_allocated_memory += new_node->allocated_size;

    new_node->parent = parent;
    if (parent != nullptr) {
        new_node->game_depth = parent->game_depth + 1;
        parent->num_children_expanded++;
    } else {
        new_node->game_depth = game_depth;
    }

    if (new_node->is_finalised) {
        for (int ii = 0; ii < sm->roleCount(); ii++) {
            const float s = new_node->getCurrentScore(ii);
            if (s > 0.99) new_node->setCurrentScore(ii, s * 1.05);
            else if (s < 0.01) new_node->setCurrentScore(ii, -0.05);
        }
        return new_node;
    }

    if (new_node->num_children == 1) return new_node;

    PuctNodeRequest req(new_node);
    scheduler->evaluate(&req);
    stats.num_evaluations++;
    total_evaluations++;
    return new_node;
}

// evaluator.cpp:216-239
PuctNode* PuctEvaluator::expandChild(PuctNode* parent, PuctNodeChild* child) {
    sm->updateBases(parent->getBaseState());
    sm->nextState(parent->moveOf(child), basestate_expand_node.data());

    const int next_depth = parent->game_depth + 1;
    child->to_node = lookupNode(basestate_expand_node.data(), next_depth);
    if (child->to_node != nullptr) {
        child->to_node->ref_count++;
        stats.num_transpositions_attached++;
        total_transpositions++;
        mirror_ok = false;   // a node with two parents: only one of them holds its mirror
    } else {
        child->unselectable = true;
        parent->unselectable_count++;
        parent->syncParent();
        child->to_node = createNode(parent, basestate_expand_node.data());
        parent->unselectable_count--;
        parent->syncParent();
        child->unselectable = false;
        child->to_node->in_parent = child;
        child->to_node->syncParent();
    }
    return child->to_node;
}

typedef std::vector<PuctNodeChild*> SortedChildren;

// evaluator.cpp:242-263: by current score of the lead role desc; unexpanded (-1) by prior desc.
// The sort runs on compact by-value keys instead of child pointers: std::sort's permutation depends
// only on the sequence of comparison results, which the keys reproduce exactly, and the keys avoid a
// dereference of every child's node per comparison.
struct SelectKey {
    float s;        // current score of the lead role, -1 when unexpanded
    float p;        // policy_prob_orig
    PuctNodeChild* c;
};
static SortedChildren sortedChildrenSelect(PuctNode* node) {
    const int n = node->num_children;
    SelectKey stack_keys[128];
    std::vector<SelectKey> heap_keys;
    SelectKey* keys = stack_keys;
    if (n > 128) {
        heap_keys.resize(n);
        keys = heap_keys.data();
    }
    for (int ii = 0; ii < n; ii++) {
        PuctNodeChild* c = node->getNodeChild(0, ii);
        keys[ii] = {c->to_node == nullptr ? -1 : c->to_node->getCurrentScore(node->lead_role_index),
                    c->policy_prob_orig, c};
    }
    std::sort(keys, keys + n, [](const SelectKey& a, const SelectKey& b) {
        if (a.s < 0 && b.s < 0) return a.p > b.p;
        return a.s > b.s;
    });
    SortedChildren children(n);
    for (int ii = 0; ii < n; ii++) children[ii] = keys[ii].c;
    return children;
}

// evaluator.cpp:266-279
static SortedChildren sortedTraversals(PuctNode* node) {
    SortedChildren children;
    for (int ii = 0; ii < node->num_children; ii++) children.push_back(node->getNodeChild(0, ii));
    auto f = [](const PuctNodeChild* a, const PuctNodeChild* b) { return a->traversals > b->traversals; };
    std::sort(children.begin(), children.end(), f);
    return children;
}

// evaluator.cpp:282-339
void PuctEvaluator::balanceFirstMoves(int max_moves) {
    GZ_ASSERT(root != nullptr);
    if (root->isTerminal()) return;
    max_moves = std::min(max_moves, (int)root->num_children);
    auto children = sortedTraversals(root);
    int wanted_traversals = -1;
    for (int ii = 0; ii < max_moves; ii++) {
        PuctNodeChild* child = children[ii];
        if (ii == 0) {
            wanted_traversals = child->traversals;
            continue;
        }
        while ((int)child->traversals < wanted_traversals) {
            PuctNode* temp_root = child->to_node;
            if (temp_root == nullptr || temp_root->isTerminal()) break;
            int worker_count = 0;
            auto f = [this, child, temp_root, &worker_count]() {
                Path path;
                path.emplace_back(this->root, child, child);
                this->treePlayout(temp_root, path);
                worker_count--;
            };
            for (int jj = 0; jj < conf->batch_size; jj++) {
                worker_count++;
                scheduler->addRunnable(f);
            }
            while (worker_count > 0) scheduler->yield();
        }
    }
}

// ---- order-independent fast paths -----------------------------------------------------------
// The reference sorts the children (std::sort, unstable) before every selection / top-visits
// choice.  Whenever the result provably does not depend on the order the sort produces -- no RNG is
// drawn inside the loop, and the winning element is strictly separated from every other element
// under the loop's own (float-truncating) comparison semantics -- a single unsorted pass returns
// the identical child.  Otherwise the literal sorted path runs.  tests/test_puct_parity.py checks
// the engine against the oracle (which always sorts); GZ_VERIFY_FASTPATH=1 cross-checks at run time.

// Process-wide switch: GZ_VERIFY_FASTPATH=1 at load, or gz_engine_set_verify_fastpath() at any
// time (a live runner can age unverified, then verify a later window).  Each fast path reads it
// once per decision, so a flip takes effect at the next selection / spin run.
static std::atomic<bool> g_verify_fastpath{[] {
    const char* e = std::getenv("GZ_VERIFY_FASTPATH");
    return e != nullptr && e[0] == '1';
}()};
// Fast-path decisions re-checked by the verification (diagnostics: a test shows the verified window
// really ran verified): one padded counter per thread slot, summed on read.
namespace {
struct alignas(64) VerifySlot {
    std::atomic<long> n{0};
};
constexpr int kVerifySlots = 256;
VerifySlot g_verified[kVerifySlots];
std::atomic<int> g_verify_next_slot{0};
struct VerifyCounter {
    std::atomic<long>* slot = &g_verified[g_verify_next_slot.fetch_add(1) % kVerifySlots].n;
};
inline void count_verified(long k = 1) { tls_instance<VerifyCounter>().slot->fetch_add(k, std::memory_order_relaxed); }
}  // namespace

static inline bool verify_fastpath() { return g_verify_fastpath.load(std::memory_order_relaxed); }

void set_verify_fastpath(bool on) { g_verify_fastpath.store(on, std::memory_order_relaxed); }
bool get_verify_fastpath() { return verify_fastpath(); }
long verified_decisions() {
    long s = 0;
    for (const VerifySlot& v : g_verified) s += v.n.load(std::memory_order_relaxed);
    return s;
}

// comparator of sortedChildrenTraversals (node.cpp:356-369, next_probability=false)
static inline bool travBefore(const PuctNodeChild* a, const PuctNodeChild* b) {
    if (a->traversals == b->traversals) return a->policy_prob > b->policy_prob;
    return a->traversals > b->traversals;
}

// chooseTopVisits (evaluator.cpp:1100-1136) as one unsorted pass: first win, first two non-losses
// and first overall under travBefore, with tie flags.  add() per child, then finish().
struct TopVisitsScan {
    const PuctNodeChild *w = nullptr, *a = nullptr, *b = nullptr, *f = nullptr;
    bool w_tie = false, f_tie = false;
    int a_n = 0, b_n = 0;

    __attribute__((always_inline)) inline void add(const PuctNodeChild* c, int ri) {
        const bool fin = c->to_node != nullptr && c->to_node->is_finalised;
        addMirrored(c, fin, fin ? c->to_node->getCurrentScore(ri) : 0.0f);
    }
    // the same with the child node's is_finalised / current score (of role ri) supplied
    __attribute__((always_inline)) inline void addMirrored(const PuctNodeChild* c, bool fin, Score sc) {
        bool win = false, loss = false;
        if (fin) {
            win = sc > 0.99;
            loss = !win && sc < 0.01;
        }
        if (f == nullptr || travBefore(c, f)) {
            f = c;
            f_tie = false;
        } else if (!travBefore(f, c)) {
            f_tie = true;
        }
        if (win) {
            if (w == nullptr || travBefore(c, w)) {
                w = c;
                w_tie = false;
            } else if (!travBefore(w, c)) {
                w_tie = true;
            }
        }
        if (!loss) {
            if (a == nullptr) {
                a = c;
                a_n = 1;
            } else if (travBefore(c, a)) {
                b = a;
                b_n = a_n;
                a = c;
                a_n = 1;
            } else if (!travBefore(a, c)) {
                a_n++;
            } else if (b == nullptr || travBefore(c, b)) {
                b = c;
                b_n = 1;
            } else if (!travBefore(b, c)) {
                b_n++;
            }
        }
    }

    // false: the sorted (exact) computation is needed
    inline bool finish(int ri, float converge_ratio, const PuctNodeChild** out) const {
        if (w != nullptr) {
            if (w_tie) return false;
            *out = w;
            return true;
        }
        if (a_n > 1 || b_n > 1) return false;   // the first two non-loss places are not unique
        if (converge_ratio > 0 && a != nullptr && b != nullptr) {
            if (a->to_node != nullptr && b->to_node != nullptr) {
                if (b->traversals > a->traversals * converge_ratio &&
                    b->to_node->getCurrentScore(ri) > a->to_node->getCurrentScore(ri))
                    *out = b;
                else
                    *out = a;
                return true;
            }
        }
        if (f == nullptr || f_tie) return false;
        *out = f;
        return true;
    }
};

bool PuctEvaluator::chooseTopVisitsFast(const PuctNode* node, const PuctNodeChild** out) const {
    TopVisitsScan scan;
    const PuctNodeChild* cs = node->children();
    for (int i = 0; i < node->num_children; ++i) scan.add(cs + i, node->lead_role_index);
    return scan.finish(node->lead_role_index, conf->top_visits_best_guess_converge_ratio, out);
}

// the first two places under sortedChildren's comparator (node.cpp:326-339, next_probability=false:
// visits desc, ties by policy_prob desc; M: visits from the mirrors) with their multiplicities, one
// pass, the comparator inlined
template <bool M>
static void top2_visits(const PuctNodeChild* cs, int n, const PuctNodeChild** pa, int* pan,
                        const PuctNodeChild** pb, int* pbn) {
    auto visits = [](const PuctNodeChild* c) -> int {
        if (c->to_node == nullptr) return 0;
        return M ? (int)c->m_visits : (int)c->to_node->visits;
    };
    // before(x, y): visits desc, ties by policy_prob desc (strict)
    const PuctNodeChild *a = cs, *b = nullptr;
    int a_n = 1, b_n = 0, av = visits(cs), bv = 0;
    for (int i = 1; i < n; ++i) {
        const PuctNodeChild* c = cs + i;
        const int cv = visits(c);
        const float cp = c->policy_prob;
        if (cv > av || (cv == av && cp > a->policy_prob)) {
            b = a; b_n = a_n; bv = av;
            a = c; a_n = 1; av = cv;
        } else if (cv == av && !(a->policy_prob > cp)) {
            a_n++;
        } else if (b == nullptr || cv > bv || (cv == bv && cp > b->policy_prob)) {
            b = c; b_n = 1; bv = cv;
        } else if (cv == bv && !(b->policy_prob > cp)) {
            b_n++;
        }
    }
    *pa = a; *pan = a_n; *pb = b; *pbn = b_n;
}

bool PuctEvaluator::convergedFast(int count, bool* out) const {
    const int n = root->num_children;
    if (n < 2) {
        *out = true;
        return true;
    }
    // one pass: the first two places under visitsBefore with their multiplicities; both must be
    // unique for the sorted order's first two elements to be order-independent
    const PuctNodeChild *a, *b;
    int a_n, b_n;
    if (mirror_ok) top2_visits<true>(root->children(), n, &a, &a_n, &b, &b_n);
    else top2_visits<false>(root->children(), n, &a, &a_n, &b, &b_n);
    if (a_n != 1 || b == nullptr || b_n != 1) return false;
    const PuctNode* n0 = a->to_node;
    const PuctNode* n1 = b->to_node;
    bool r = false;
    if (n0 != nullptr && n1 != nullptr) {
        const int role_index = root->lead_role_index;
        r = n0->getCurrentScore(role_index) > n1->getCurrentScore(role_index) && n0->visits > n1->visits + count;
    }
    *out = r;
    return true;
}

// comparator of sortedChildrenSelect (evaluator.cpp:242-263)
static inline bool selectBefore(const PuctNodeChild* a, const PuctNodeChild* b, int lead) {
    const float sa = a->to_node == nullptr ? -1 : a->to_node->getCurrentScore(lead);
    const float sb = b->to_node == nullptr ? -1 : b->to_node->getCurrentScore(lead);
    if (sa < 0 && sb < 0) return a->policy_prob_orig > b->policy_prob_orig;
    return sa > sb;
}

// Unsorted selection; returns false when the literal sorted loop must run instead (the RNG is then
// left exactly as it was on entry).
//
// Root latch (evaluator.cpp:461-475): at the root with 1000 < visits < 4e7 the reference draws
// rng.get() once for every child that reaches the latch test, in sortedChildrenSelect order, and a
// child is skipped when its draw is > 0.1 and its traversals exceed 16 and 0.66 * visits.  At most
// one child d can exceed 0.66 * visits (traversals sum to at most visits), so only d's draw matters:
// its position in the sorted order is the number of reaching children that sort strictly before it,
// which is order-independent unless another reaching child ties with d under the comparator (then
// the literal path runs).  The draws are made in the same number, d's is the one at that position.
// ---- child selection --------------------------------------------------------------------------
// Per-thread scratch of the selection pass (every evaluator of a thread runs on that thread; nothing
// here is live across a coroutine switch).
namespace {
struct SelectScratch {
    std::vector<double> base, expl, inflight, scores;
    std::vector<uint32_t> trav;
    std::vector<float> pcp;          // puct_constant * policy_prob (float, as the reference's product)
    std::vector<int32_t> tr1;        // traversals + 1 (the exploration term's int)
    std::vector<uint8_t> kind, bcs;
    std::vector<float> key_s, key_p;
    // sortedChildrenSelect permutation cache, keyed by the sort's input keys only: std::sort's
    // permutation is a function of the sequence of comparison outcomes, hence of the keys
    std::vector<float> cached_s, cached_p;
    std::vector<uint16_t> perm, perm2;
    std::vector<uint8_t> mark;
    int cached_n = -1;
    struct Key {
        float s, p;
        uint16_t i;
    };
    std::vector<Key> tmp;

    void reserve(int n) {
        if ((int)base.size() >= n) return;
        // (expl / pcp / tr1 / inflight padded to whole 4-lane vectors: explorationTerms)
        const int n4 = (n + 3) & ~3;
        base.resize(n); expl.resize(n4); inflight.resize(n4); scores.resize(n); trav.resize(n);
        pcp.resize(n4); tr1.resize(n4);
        kind.resize(n); bcs.resize(n); key_s.resize(n); key_p.resize(n); perm.resize(n); tmp.resize(n);
        perm2.resize(n); mark.resize(n);
        cached_s.resize(n); cached_p.resize(n);
    }

    const uint16_t* sortedOrder(int n) {
        if (n == cached_n && std::memcmp(key_s.data(), cached_s.data(), n * sizeof(float)) == 0 &&
            std::memcmp(key_p.data(), cached_p.data(), n * sizeof(float)) == 0)
            return perm.data();
        for (int i = 0; i < n; ++i) tmp[i] = Key{key_s[i], key_p[i], (uint16_t)i};
        std::sort(tmp.begin(), tmp.begin() + n, [](const Key& a, const Key& b) {
            if (a.s < 0 && b.s < 0) return a.p > b.p;
            return a.s > b.s;
        });
        for (int i = 0; i < n; ++i) perm[i] = tmp[i].i;
        std::memcpy(cached_s.data(), key_s.data(), n * sizeof(float));
        std::memcpy(cached_p.data(), key_p.data(), n * sizeof(float));
        cached_n = n;
        return perm.data();
    }
};

// child kinds of the selection pass
enum : uint8_t { kSkip = 0, kPrior = 1, kScored = 2, kWinReturn = 3, kBad = 4 };
}  // namespace

// expl[i] = (double)pcp[i] * sqrt_node_visits / ((double)tr1[i] + inflight[i]) for every child, four
// at a time (one packed division per four children instead of four scalar ones: the selection pass
// was bound by the divider), tr1[i] == 0 marking a zero term (a finalised child that is neither a win
// nor a loss).  The reference's expression `puct_constant * policy_prob * sqrt_node_visits /
// (traversals + inflight_visits)` is float * float (rounded to float), then * double, then / (int +
// double): exactly these IEEE operations per lane.  (Padded lanes compute garbage nobody reads.)
static inline void explorationTerms(const float* pcp, const int32_t* tr1, const double* inflight, double sq,
                                    double* expl, int n) {
    const __m256d sq4 = _mm256_set1_pd(sq);
    const __m256d zero = _mm256_setzero_pd();
    for (int i = 0; i < n; i += 4) {
        const __m128i t = _mm_loadu_si128((const __m128i*)(tr1 + i));
        const __m256d num = _mm256_mul_pd(_mm256_cvtps_pd(_mm_loadu_ps(pcp + i)), sq4);
        const __m256d den = _mm256_add_pd(_mm256_cvtepi32_pd(t), _mm256_loadu_pd(inflight + i));
        const __m256d q = _mm256_div_pd(num, den);
        const __m256d z = _mm256_castsi256_pd(_mm256_cvtepi32_epi64(_mm_cmpeq_epi32(t, _mm_setzero_si128())));
        _mm256_storeu_pd(expl + i, _mm256_blendv_pd(q, zero, z));
    }
}

// The literal selection loop of the reference over sortedChildrenSelect (evaluator.cpp:341-517),
// kept verbatim for the verification mode (GZ_VERIFY_FASTPATH=1) and for nodes with > 65535
// children.  Returns the chosen child (or null) and its best-score companion in *best_out.
PuctNodeChild* PuctEvaluator::selectChildLiteral(PuctNode* node, int depth, float prior_score,
                                                 double sqrt_node_visits, PuctNodeChild** best_out) {
    float best_score = -1;
    PuctNodeChild* best_child = nullptr;
    float best_child_score_actual_score = -1;
    PuctNodeChild* best_child_score = nullptr;
    PuctNodeChild* bad_fallback = nullptr;
    float best_fallback_score = -1;
    PuctNodeChild* best_fallback = nullptr;
    int unselectables = 0;

    SortedChildren children = sortedChildrenSelect(node);
    for (PuctNodeChild* c : children) {
        if (c->unselectable) {
            unselectables++;
            continue;
        } else if (c->to_node != nullptr && (c->to_node->num_children > 0 &&
                                             c->to_node->unselectable_count == c->to_node->num_children)) {
            unselectables++;
            continue;
        }

        double child_score = prior_score;
        const int traversals = c->traversals + 1;
        const double inflight_visits = c->to_node != nullptr ? c->to_node->inflight_visits : 0;
        double exploration_score = node->puct_constant * c->policy_prob * sqrt_node_visits /
                                   (traversals + inflight_visits);

        if (c->to_node != nullptr) {
            PuctNode* cn = c->to_node;
            child_score = cn->getCurrentScore(node->lead_role_index);
            if (cn->is_finalised) {
                if (child_score > 0.99) {
                    if (depth > 0) {
                        *best_out = c;
                        return c;
                    }
                    child_score *= 1.0f + node->puct_constant;
                } else if (child_score < 0.01) {
                    bad_fallback = c;
                    continue;
                } else {
                    exploration_score = 0.0;
                }
            }
            if ((cn->is_finalised || cn->visits > 42) && child_score > best_child_score_actual_score) {
                best_child_score_actual_score = child_score;
                best_child_score = c;
            }
        }

        if (c->traversals > 0 && inflight_visits > 0) {
            const double discounted_visits = inflight_visits * (rng.get() + 0.5);
            child_score = (child_score * c->traversals) / (c->traversals + discounted_visits);
        }

        const float limit_latch_root = 0.66;
        node->coldOf(c).debug_node_score = child_score;
        node->coldOf(c).debug_puct_score = exploration_score;
        const double score = child_score + exploration_score;

        if (node->visits > 1000 && node->visits < 40000000 && depth == 0 && rng.get() > 0.1) {
            if (c->traversals > 16 && c->traversals > node->visits * limit_latch_root) {
                if (best_fallback == nullptr || score > best_fallback_score) {
                    best_fallback = c;
                    best_fallback_score = score;
                }
                continue;
            }
        }

        if (score > best_score) {
            best_child = c;
            best_score = score;
        }
    }

    if (best_child == nullptr) {
        if (best_fallback != nullptr) {
            best_child = best_child_score != nullptr ? best_child_score : best_fallback;
        } else if (bad_fallback != nullptr) {
            if (unselectables > 0) scheduler->yield();
            best_child = bad_fallback;
        } else {
            stats.num_blocked++;
        }
    }
    if (best_child_score == nullptr) best_child_score = best_child;
    *best_out = best_child_score;
    return best_child;
}

// selectChild (evaluator.cpp:341-517).  One pass over the children gathers everything the
// reference computes from them: priorScore's chooseTopVisits scan and FPU policy sum
// (evaluator.cpp:1195-1224), each child's selection terms and its sort key.  Then:
//   1. when the winner provably does not depend on the order the reference's std::sort produces
//      (no RNG-dependent step, strictly separated maximum), it is returned directly;
//   2. otherwise the reference's loop runs over the gathered arrays in sortedChildrenSelect order,
//      with the permutation recomputed only when a sort key changed (in the spinning phases of
//      self-play -- the root re-selecting finalised children -- the keys repeat for thousands of
//      playouts); RNG draws (inflight discount, root latch) happen exactly as in the reference.
PuctNodeChild* PuctEvaluator::selectChild(PuctNode* node, Path& path) {
    GZ_ASSERT(!node->isTerminal());
    const int depth = (int)path.size();
    setPuctConstant(node, depth);

    if (node->num_children == 1) {
        PuctNodeChild* child = node->getNodeChild(0, 0);
        path.emplace_back(node, child, child);
        return child;
    }

    if (depth == 0) setDirichletNoise(node);

    const double sqrt_node_visits = std::sqrt(node->visits + 1);
    const int n = node->num_children;

    // Forced reply (depth > 0): the reference returns the first finalised child scoring > 0.99 for
    // the node's lead role in sortedChildrenSelect order (evaluator.cpp:415-424); with a unique
    // highest-scoring such child, no tie among them and no RNG draw before it (the inflight
    // discount, :441-444), that child is the result whatever else the node holds.  Deep in an
    // NN-free spin (a solved endgame: every playout a forced line to a terminal) this is the common
    // interior node: one light pass over the mirrors instead of the full selection pass.
    if (depth > 0 && mirror_ok && n <= 65535) {
        const PuctNodeChild* cs0 = node->children();
        int fw = -1;
        float fk = 0.f;
        bool tied = false, draws = false;
        for (int i = 0; i < n; ++i) {
            const PuctNodeChild* c = cs0 + i;
            if (c->to_node == nullptr || c->unselectable) continue;
            if (c->m_inflight != 0 && c->traversals > 0) draws = true;
            if ((c->m_flags & (kMirrorFinalised | kMirrorAllUnselectable)) != kMirrorFinalised) continue;
            const float k = c->m_score;
            if (!((double)k > 0.99)) continue;
            if (fw < 0 || k > fk) {
                fw = i;
                fk = k;
                tied = false;
            } else if (k == fk) {
                tied = true;
            }
        }
        if (fw >= 0 && tied && !draws) {
            // tied wins: the entry of the last sorted decision, while it holds (ForcedEntry)
            const ForcedEntry& fe = forced_cache[forcedSlot(node)];
            if (fe.node == node && fe.nch == n) {
                const PuctNodeChild* c = cs0 + fe.child;
                if (node->visits - fe.visits == c->traversals - fe.trav && c->m_score == fk &&
                    (c->m_flags & (kMirrorFinalised | kMirrorAllUnselectable)) == kMirrorFinalised && !c->unselectable) {
                    fw = fe.child;
                    tied = false;
                }
            }
        }
        if (fw >= 0 && !tied && !draws) {
            PuctNodeChild* chosen = node->getNodeChild(0, fw);
            if (verify_fastpath()) {
                const Rng rng_before = rng;
                PuctNodeChild* lit_best = nullptr;
                PuctNodeChild* lit = selectChildLiteral(node, depth, priorScore(node, depth), sqrt_node_visits, &lit_best);
                if (lit != chosen || !(rng == rng_before)) {
                    std::fprintf(stderr, "gz forced-reply verification mismatch (depth %d, n %d)\n", depth, n);
                    std::abort();
                }
                count_verified();
            }
            sd(kSdSelectForced);
            path.emplace_back(node, chosen, chosen);
            return chosen;
        }
    }
    if (n > 65535) {
        PuctNodeChild* best = nullptr;
        PuctNodeChild* chosen = selectChildLiteral(node, depth, priorScore(node, depth), sqrt_node_visits, &best);
        if (chosen != nullptr) path.emplace_back(node, chosen, best);
        return chosen;
    }

    PuctNodeChild* cs = node->children();
    {   // the pass below streams the whole child array: request every line of it up front (the
        // array is usually cold -- hundreds of games' trees per thread -- and its lines are
        // independent, so their misses overlap instead of trickling in behind the loop)
        const char* p0 = reinterpret_cast<const char*>(cs);
        const char* p1 = reinterpret_cast<const char*>(cs + n);
        for (const char* q = p0; q < p1; q += 64) __builtin_prefetch(q, 1, 3);
    }
    SelectScratch& S = tls_instance<SelectScratch>();
    S.reserve(n);
    const int lead = node->lead_role_index;
    const bool latch = node->visits > 1000 && node->visits < 40000000 && depth == 0;
    const float limit_latch_root = 0.66;

    const bool want_top = node->visits > 8;
    TopVisitsScan top;
    float total_policy_visited = 0.0;
    int win = -1;
    bool win_tied = false, rng_steps = false;
    float win_key = 0.f;
    int latch_d = -1, latch_count = 0, reach = 0;
    const bool M = mirror_ok;   // read the children's mirrors (node.h) instead of their nodes
    for (int i = 0; i < n; ++i) {
        PuctNodeChild* c = cs + i;
        const PuctNode* cn = c->to_node;
        // the child node's fields this pass reads
        uint32_t cn_visits = 0;
        float cn_score = -1;
        uint16_t cn_inflight = 0;
        uint8_t cn_flags = 0;
        if (cn != nullptr) {
            if (M) {
                cn_visits = c->m_visits;
                cn_score = c->m_score;
                cn_inflight = c->m_inflight;
                cn_flags = c->m_flags;
            } else {
                cn_visits = cn->visits;
                cn_score = cn->getCurrentScore(lead);
                cn_inflight = cn->inflight_visits;
                cn_flags = (uint8_t)((cn->is_finalised ? kMirrorFinalised : 0) |
                                     (cn->num_children > 0 && cn->unselectable_count == cn->num_children
                                          ? kMirrorAllUnselectable : 0));
            }
        }
        const bool cn_final = (cn_flags & kMirrorFinalised) != 0;
        if (want_top) top.addMirrored(c, cn != nullptr && cn_final, cn_score);
        if (cn != nullptr && cn_visits > 0) total_policy_visited += c->policy_prob;
        S.key_s[i] = cn == nullptr ? -1 : cn_score;
        S.key_p[i] = c->policy_prob_orig;

        S.kind[i] = kSkip;
        // the exploration term's factors; the term itself, node->puct_constant * policy_prob *
        // sqrt_node_visits / (traversals + 1 + inflight), for every child at once after the pass
        // (explorationTerms: packed divisions, the same IEEE operations in the same order)
        const double inflight_visits = cn != nullptr ? cn_inflight : 0;
        S.pcp[i] = node->puct_constant * c->policy_prob;
        S.tr1[i] = (int32_t)(c->traversals + 1);
        S.inflight[i] = inflight_visits;
        if (c->unselectable) continue;
        if (cn != nullptr && (cn_flags & kMirrorAllUnselectable)) continue;
        bool zero_expl = false;
        S.trav[i] = c->traversals;
        if (c->traversals > 0 && inflight_visits > 0) rng_steps = true;   // discount draws RNG
        if (cn != nullptr) {
            double child_score = cn_score;
            if (cn_final) {
                if (child_score > 0.99) {
                    if (depth > 0) {
                        // the first win in sortedChildrenSelect order has the highest current score
                        S.kind[i] = kWinReturn;
                        const float k = cn_score;
                        if (win < 0 || k > win_key) {
                            win = i;
                            win_key = k;
                            win_tied = false;
                        } else if (k == win_key) {
                            win_tied = true;
                        }
                        continue;
                    }
                    child_score *= 1.0f + node->puct_constant;
                } else if (child_score < 0.01) {
                    S.kind[i] = kBad;   // bad_fallback candidate
                    continue;
                } else {
                    zero_expl = true;
                }
            }
            S.kind[i] = kScored;
            S.base[i] = child_score;
            S.bcs[i] = cn_final || cn_visits > 42;
        } else {
            S.kind[i] = kPrior;
        }
        if (zero_expl) S.tr1[i] = 0;   // a finalised non-win child: exploration 0 (marked, set below)
        ++reach;
        if (latch && c->traversals > 16 && c->traversals > node->visits * limit_latch_root) {
            ++latch_count;
            latch_d = i;
        }
    }

    explorationTerms(S.pcp.data(), S.tr1.data(), S.inflight.data(), sqrt_node_visits, S.expl.data(), n);

    // priorScore (evaluator.cpp:1195-1224)
    float prior_score = node->getFinalScore(lead);
    if (want_top) {
        const PuctNodeChild* best_top = nullptr;
        if (!top.finish(lead, conf->top_visits_best_guess_converge_ratio, &best_top)) best_top = chooseTopVisitsExact(node);
        if (best_top->to_node != nullptr) prior_score = best_top->to_node->getCurrentScore(lead);
    }
    {
        float fpu_reduction = depth == 0 ? conf->fpu_prior_discount_root : conf->fpu_prior_discount;
        if (fpu_reduction > 0) {
            fpu_reduction *= std::sqrt(total_policy_visited);
            prior_score -= fpu_reduction;
        }
    }

    const bool verify = verify_fastpath();
    const Rng rng_before = rng;
    PuctNodeChild* chosen = nullptr;
    PuctNodeChild* chosen_best = nullptr;
    bool done = false;

    // 1. order-independent outcome
    if (win >= 0) {
        if (!win_tied && !rng_steps) {
            chosen = chosen_best = cs + win;
            done = true;
        }
    } else if (!rng_steps && latch_count <= 1) {
        // scores and the three best candidates (enough to decide strict separation both for the
        // full candidate set and for the set without the latch candidate d)
        int i1 = -1, i2 = -1, i3 = -1;
        double v1 = 0.0, v2 = 0.0, v3 = 0.0;
        for (int i = 0; i < n; ++i) {
            if (S.kind[i] != kPrior && S.kind[i] != kScored) {
                S.scores[i] = -1e300;   // not a candidate
                continue;
            }
            const double child_score = S.kind[i] == kPrior ? (double)prior_score : S.base[i];
            const double score = child_score + S.expl[i];
            S.scores[i] = score;
            // ties keep the earlier index first; separation below rejects near-ties anyway
            if (i1 < 0 || score > v1) {
                i3 = i2; v3 = v2;
                i2 = i1; v2 = v1;
                i1 = i; v1 = score;
            } else if (i2 < 0 || score > v2) {
                i3 = i2; v3 = v2;
                i2 = i; v2 = score;
            } else if (i3 < 0 || score > v3) {
                i3 = i; v3 = score;
            }
        }
        // order independence of `if (score > best_score_float)`: the max m must replace any
        // incumbent (m > float(c)) and never be replaced (c <= float(m)); float rounding is
        // monotone, so checking the runner-up suffices
        auto separated = [](int ib, double vb, int ir, double vr) {
            if (ib < 0 || !(vb > -1.0)) return false;
            if (ir < 0) return true;
            const double fm = (float)vb;
            return !(vr > fm) && vb > (double)(float)vr;
        };
        const bool sep_all = separated(i1, v1, i2, v2);
        int j1 = i1, j2 = i2;
        double w1 = v1, w2 = v2;
        if (latch_d >= 0) {   // the set without d
            if (i1 == latch_d) { j1 = i2; w1 = v2; j2 = i3; w2 = v3; }
            else if (i2 == latch_d) { j2 = i3; w2 = v3; }
        }
        const bool sep_no_d = latch_d >= 0 && separated(j1, w1, j2, w2);

        bool ok = sep_all || sep_no_d;
        int best = i1;
        if (ok && latch) {
            // root latch: only d's draw matters; its rank among the reaching children in sorted
            // order must be determined without the sort (no reaching child ties with d)
            int rank = 0;
            if (latch_d >= 0) {
                if (reach < 2) ok = false;   // d alone: the fallback rules decide
                const float ds = S.key_s[latch_d], dp = S.key_p[latch_d];
                for (int i = 0; ok && i < n; ++i) {
                    if (i == latch_d || S.scores[i] == -1e300) continue;
                    const float is = S.key_s[i], ip = S.key_p[i];
                    const bool i_before = (is < 0 && ds < 0) ? ip > dp : is > ds;
                    const bool d_before = (ds < 0 && is < 0) ? dp > ip : ds > is;
                    if (i_before) ++rank;
                    else if (!d_before) ok = false;   // tie: position undetermined
                }
            } else if (!sep_all) {
                ok = false;
            }
            if (ok) {
                // one draw per reaching child; only d's (at `rank`) is read
                bool latched = false;
                if (latch_d >= 0) {
                    rng.discard((uint64_t)rank);
                    latched = rng.get() > 0.1;
                    rng.discard((uint64_t)(reach - rank - 1));
                } else {
                    rng.discard((uint64_t)reach);
                }
                if (latched) {
                    ok = sep_no_d;
                    best = j1;
                } else {
                    ok = sep_all;
                }
            }
        } else if (ok) {
            ok = sep_all;
        }
        if (ok) {
            chosen = chosen_best = cs + best;
            done = true;
        } else {
            rng = rng_before;
        }
    }

    // 2. the reference's loop in sorted order over the gathered terms
    sd(kSdSelect);
    if (!done) {
        sd(kSdSelectSorted);
        const uint16_t* order = S.sortedOrder(n);
        float best_score = -1;
        PuctNodeChild* best_child = nullptr;
        float best_child_score_actual_score = -1;
        PuctNodeChild* best_child_score = nullptr;
        PuctNodeChild* bad_fallback = nullptr;
        float best_fallback_score = -1;
        PuctNodeChild* best_fallback = nullptr;
        int unselectables = 0;
        bool returned = false;
        for (int k = 0; k < n; ++k) {
            const int i = order[k];
            PuctNodeChild* c = cs + i;
            const uint8_t kd = S.kind[i];
            if (kd == kSkip) {
                unselectables++;
                continue;
            }
            if (kd == kWinReturn) {
                chosen = chosen_best = c;
                returned = true;
                if (depth > 0 && mirror_ok && !rng_steps) {   // (ForcedEntry: tied wins decided by the sort)
                    ForcedEntry& fe = forced_cache[forcedSlot(node)];
                    fe.node = node;
                    fe.visits = node->visits;
                    fe.trav = c->traversals;
                    fe.child = (uint16_t)i;
                    fe.nch = (uint16_t)n;
                }
                break;
            }
            if (kd == kBad) {
                bad_fallback = c;
                continue;
            }
            double child_score = kd == kPrior ? (double)prior_score : S.base[i];
            const double exploration_score = S.expl[i];
            if (kd == kScored && S.bcs[i] && child_score > best_child_score_actual_score) {
                best_child_score_actual_score = child_score;
                best_child_score = c;
            }
            const double inflight_visits = S.inflight[i];
            const uint32_t trav = S.trav[i];
            if (trav > 0 && inflight_visits > 0) {
                const double discounted_visits = inflight_visits * (rng.get() + 0.5);
                child_score = (child_score * trav) / (trav + discounted_visits);
            }
            PuctChildCold& cc = node->cold()[i];
            cc.debug_node_score = child_score;
            cc.debug_puct_score = exploration_score;
            const double score = child_score + exploration_score;
            if (latch && rng.get() > 0.1) {
                if (trav > 16 && trav > node->visits * limit_latch_root) {
                    if (best_fallback == nullptr || score > best_fallback_score) {
                        best_fallback = c;
                        best_fallback_score = score;
                    }
                    continue;
                }
            }
            if (score > best_score) {
                best_child = c;
                best_score = score;
            }
        }
        if (!returned) {
            if (best_child == nullptr) {
                if (best_fallback != nullptr) {
                    best_child = best_child_score != nullptr ? best_child_score : best_fallback;
                } else if (bad_fallback != nullptr) {
                    if (unselectables > 0) scheduler->yield();
                    best_child = bad_fallback;
                } else {
                    stats.num_blocked++;
                }
            }
            if (best_child_score == nullptr) best_child_score = best_child;
            chosen = best_child;
            chosen_best = best_child_score;
        }
    }

    if (verify) {
        // replay the literal reference loop from the same RNG state: same child, same RNG state
        const Rng rng_after = rng;
        rng = rng_before;
        const float exact_prior = priorScore(node, depth);
        PuctNodeChild* lit_best = nullptr;
        PuctNodeChild* lit = selectChildLiteral(node, depth, exact_prior, sqrt_node_visits, &lit_best);
        if (!(exact_prior == prior_score) || lit != chosen || !(rng == rng_after)) {
            std::fprintf(stderr, "gz selectChild verification mismatch (depth %d, n %d)\n", depth, n);
            std::abort();
        }
        count_verified();
    }
    if (chosen != nullptr) path.emplace_back(node, chosen, chosen_best);
    return chosen;
}

// evaluator.cpp:519-656
void PuctEvaluator::backup(float* new_scores, const Path& path) {
    const int role_count = sm->roleCount();
    auto forceFinalise = [role_count](PuctNode* cur) -> const PuctNodeChild* {
        float best_score = -1;
        const PuctNodeChild* best = nullptr;
        bool more_to_explore = false;
        for (int ii = 0; ii < cur->num_children; ii++) {
            const PuctNodeChild* c = cur->getNodeChild(role_count, ii);
            if (c->to_node != nullptr && c->to_node->is_finalised) {
                const float score = c->to_node->getCurrentScore(cur->lead_role_index);
                if (score > 0.99) return c;
                if (score > best_score) {
                    best_score = score;
                    best = c;
                }
            } else {
                more_to_explore = true;
            }
        }
        return more_to_explore ? nullptr : best;
    };

    bool bp_finalised_only_once = conf->backup_finalised;
    for (int index = (int)path.size() - 1; index >= 0; index--) {
        const PathElement& cur = path[index];
        if (bp_finalised_only_once && !cur.node->is_finalised && cur.node->lead_role_index >= 0) {
            bp_finalised_only_once = false;
            const PuctNodeChild* finalised_child = forceFinalise(cur.node);
            if (finalised_child != nullptr) {
                for (int ii = 0; ii < role_count; ii++)
                    cur.node->setCurrentScore(ii, finalised_child->to_node->getCurrentScore(ii));
                cur.node->is_finalised = true;
            }
        }

        if (cur.node->is_finalised) {
            for (int ii = 0; ii < role_count; ii++) new_scores[ii] = cur.node->getCurrentScore(ii);
        } else {
            for (int ii = 0; ii < role_count; ii++) {
                float visits = cur.node->visits;
                if (visits > 100000) visits = 100000 + 0.1f * (visits - 100000);
                const float score = ((visits * cur.node->getCurrentScore(ii) + new_scores[ii]) / (visits + 1.0f));
                cur.node->setCurrentScore(ii, score);
            }
        }

        cur.node->visits++;
        if (cur.node->inflight_visits > 0) cur.node->inflight_visits--;
        cur.node->syncParent();

        if (cur.choice != nullptr) {
            cur.choice->traversals++;
            if (cur.node->visits > 23) {
                const float cur_score = cur.node->getCurrentScore(cur.node->lead_role_index);
                float apply, minimum;
                if (cur_score > 0.3 && cur_score < 0.7) {
                    apply = 0.995;
                    minimum = 0.02f;
                } else if (cur_score > 0.15 && cur_score < 0.85) {
                    apply = 0.9975;
                    minimum = 0.03f;
                } else {
                    apply = 0.9975;
                    minimum = 0.10f;
                }
                if (cur.choice->policy_prob > minimum) {
                    cur.choice->policy_prob *= apply;
                    cur.choice->policy_prob = std::max(minimum, cur.choice->policy_prob);
                }
            }
        }

        if (cur.node->visits % 100 == 0) cur.node->normaliseX();
    }
}

// evaluator.cpp:658-720
int PuctEvaluator::treePlayout(PuctNode* current, Path& path) {
    GZ_ASSERT(current != nullptr && !current->isTerminal());
    float scores[kMaxRoles];
    PuctNodeChild* child = nullptr;

    while (true) {
        if (current->isTerminal()) {
            path.emplace_back(current, nullptr, nullptr);
            break;
        }
        if (current->is_finalised) {
            path.emplace_back(current, nullptr, nullptr);
            break;
        }
        while (true) {
            child = selectChild(current, path);
            if (child != nullptr) break;
            scheduler->yield();
        }
        if (child->to_node == nullptr) {
            current = expandChild(current, child);
            if (current->is_finalised || current->num_children > 1) {
                path.emplace_back(current, nullptr, nullptr);
                break;
            }
        }
        current->inflight_visits++;
        current->syncParent();
        current = child->to_node;
    }

    if (current->is_finalised) stats.playouts_finals++;
    for (int ii = 0; ii < sm->roleCount(); ii++) scores[ii] = current->getCurrentScore(ii);
    backup(scores, path);
    stats.num_tree_playouts++;
    total_tree_playouts++;
    return (int)path.size();
}

// ---- root spin fast path ------------------------------------------------------------------------
// With two or more finalised winning children at the root, the reference's playout loop is never
// "converged" (the two most visited children are wins with equal scores) and runs until enough NN
// evaluations accumulate -- up to millions of playouts per move, nearly all of them root -> win ->
// backup with no evaluation (playoutMain, evaluator.cpp:744-886).  Such a playout only needs the
// scores of the few children that can still win the selection: spinRun runs playouts of
// that form with the reference's arithmetic and RNG consumption (the root-latch draw per reaching
// child), and returns false whenever the proof below does not hold or another child wins the
// selection, after which the ordinary treePlayout runs.
//
// An epoch (spinBuild, one pass over the children) establishes, for root visits v in [v0, v_end):
//   * no child is in flight, none is unselectable or being expanded, the Dirichlet noise cannot
//     change, backup_finalised is off (the root cannot become finalised), no child can reach the
//     root-latch threshold except the wins (checked per playout);
//   * every other candidate i scores at most U_i = base_i + (float)(pc(v_end-1) * p_i) *
//     sqrt(v_end) / (t_i + 1), the value its exploration term reaches at the epoch's last playout
//     (pc and sqrt increase with v; its traversals and policy_prob do not change while it is not
//     selected, and normaliseX -- every 100 root visits -- ends the epoch), with base_i its current
//     score, or for unexpanded children the FPU prior, bounded by the top win's score;
//   * candidates whose bound reaches the wins' floor min_w s_w * (1 + pc(v0)) are WATCHED: scored
//     exactly every playout (an unexpanded one with the exact FPU prior, whose policy sum is folded
//     over the visited children in index order as the reference does);
//   * the two most visited children are wins with equal scores, so converged() is false for the
//     whole epoch (only wins gain visits) -- or playoutMain evaluates it as usual.
// Per playout the wins and watched candidates are scored in sortedChildrenSelect order (constant in
// the epoch: no sort key changes) with the reference loop's `score > best_score` (float) semantics;
// the result stands when it is a win and beats every unwatched bound with margin (unwatched
// elements below the final best cannot change the loop's outcome).


// GZ_SPIN_FAST=0: no spin fast path; =2: the fast path without spinRunRegs (tests compare all three)
static int spin_fast_mode() {
    static const int v = [] {
        const char* e = std::getenv("GZ_SPIN_FAST");
        return e == nullptr || e[0] == '\0' ? 1 : std::atoi(e);
    }();
    return v;
}
static bool spin_fast_enabled() { return spin_fast_mode() != 0; }

static inline double spin_margin_up(double x) { return x + std::fabs(x) * 1e-6 + 1e-12; }
// the largest policy rescaling (relative, per normalisation; twice that cumulated) an epoch's bounds
// absorb: well inside the bounds' 1e-6 relative margin
constexpr double kSpinDrift = 2e-7;
static inline double spin_margin_down(double x) { return x - std::fabs(x) * 1e-6 - 1e-12; }

bool PuctEvaluator::spinBuild() {
    sd(kSdBuilds);
    spin.valid = false;
    PuctNode* node = root;
    const int lead = node->lead_role_index;
    if (conf->backup_finalised || conf->think_time > 0 || node->is_finalised || node->isTerminal() ||
        node->num_children < 2 || node->visits <= 8 || node->inflight_visits != 0 || lead < 0 ||
        (!node->dirichlet_noise_set && conf->dirichlet_noise_pct >= 0 && node->getCurrentScore(lead) <= 0.95)) {
        sd(kSdFailRoot);
        return false;
    }

    const uint32_t v0 = node->visits;
    PuctNodeChild* cs = node->children();
    const int n = node->num_children;
    // One pass over the children gathers what the epoch needs into the thread's scratch (from their
    // mirrors in the child array, node.h, while those are exact: one streamed array instead of one
    // cold node per child): the sort keys, and the non-win candidates' selection terms.
    const bool M = mirror_ok;
    SelectScratch& S = tls_instance<SelectScratch>();
    S.reserve(n);
    enum : uint8_t { kUnexp = 0, kWinC = 1, kOther = 2, kSkipC = 3 };
    uint8_t* kind = S.kind.data();   // (reused: the selection pass's kinds are dead here)
    int nw = 0, reach = 0, nvis = 0, nother = 0;
    uint16_t* other = S.perm2.data();   // non-win candidates
    bool regs_ok = true;
    float win_score = 0.f;
    uint32_t wv0 = 0, wv1 = 0;   // the two largest win visit counts
    uint32_t nonwin_max_visits = 0;
    bool have_nonwin_visits = false;
    for (int i = 0; i < n; ++i) {
        const PuctNodeChild* c = cs + i;
        const PuctNode* cn = c->to_node;
        if (c->unselectable) return sd(kSdFailUnselectable), false;
        S.key_p[i] = c->policy_prob_orig;
        if (cn == nullptr) {
            S.key_s[i] = -1;
            kind[i] = kUnexp;
        } else {
            uint32_t visits;
            float score;
            uint16_t inflight;
            bool finalised, all_unsel;
            if (M) {
                visits = c->m_visits;
                score = c->m_score;
                inflight = c->m_inflight;
                finalised = (c->m_flags & kMirrorFinalised) != 0;
                all_unsel = (c->m_flags & kMirrorAllUnselectable) != 0;
            } else {
                visits = cn->visits;
                score = cn->getCurrentScore(lead);
                inflight = cn->inflight_visits;
                finalised = cn->is_finalised;
                all_unsel = cn->num_children > 0 && cn->unselectable_count == cn->num_children;
            }
            S.key_s[i] = score;
            S.base[i] = score;
            if (visits > 0) {
                if (nvis == SpinEpoch::kMaxVisited) return sd(kSdFailVisited), false;
                spin.visited[nvis++] = (uint16_t)i;
            }
            if (inflight != 0 || all_unsel) return sd(kSdFailInflight), false;
            kind[i] = kOther;
            S.bcs[i] = finalised;
            if (finalised) {
                if (score > 0.99) {
                    if (!cn->isTerminal() || nw == SpinEpoch::kMaxWins) return sd(kSdFailWinNode), false;
                    if (nw > 0 && !(score == win_score)) return sd(kSdFailWinScore), false;
                    regs_ok = regs_ok && cn->num_children == 0;
                    win_score = score;
                    ++nw;
                    if (visits >= wv0) { wv1 = wv0; wv0 = visits; }
                    else if (visits > wv1) wv1 = visits;
                    ++reach;
                    kind[i] = kWinC;
                    continue;
                }
                if (score < 0.01) {   // bad_fallback candidate: never reached while a candidate exists
                    kind[i] = kSkipC;
                    continue;
                }
            }
            have_nonwin_visits = true;
            nonwin_max_visits = std::max(nonwin_max_visits, visits);
        }
        // a non-win candidate: the latch threshold only gets further away as v grows (checked
        // whether or not the latch is active yet: it may become active inside the epoch)
        if (c->traversals > 16 && c->traversals > node->visits * 0.66f) return sd(kSdFailLatch), false;
        ++reach;
        other[nother++] = (uint16_t)i;
    }
    if (nw < 2) return sd(kSdFailFewWins), false;
    // converged() (evaluator.cpp:1342-1362) compares the two most visited children: both wins with
    // equal scores -> false, and it stays false while only wins gain visits; otherwise playoutMain
    // evaluates it as usual
    const bool conv_false = !(have_nonwin_visits && !(nonwin_max_visits < wv1));

    // the FPU prior of unexpanded children: the top-visits child is a win (chooseTopVisits returns
    // the first win), so prior = win score - fpu * sqrt(...) <= win score
    const double prior_bound = (double)win_score;
    auto pc_at = [&](uint32_t v) {
        float p = puct_log(v);
        p += conf->puct_constant_root;
        return p;
    };
    // the best win scores at least its child_score = s_w * (1 + pc(v)) >= s_w * (1 + pc(v0))
    double floor_win = win_score;
    floor_win *= 1.0f + pc_at(v0);
    const double floor_adj = spin_margin_down(floor_win);

    uint8_t* watched = S.mark.data();
    // Epoch length.  The bounds read the children's policies, which change at normaliseX (every
    // 100 root visits).  Deep in a spin that rescales every policy by 1 / total with total within
    // a few float ulps of 1 (the wins sit below their decay minimum), and the spin loops re-check
    // the factor at each normalisation, ending the epoch when it drifts (kSpinDrift): so a long
    // epoch (16 normalisations) is tried first and taken when it leaves every non-win unwatched;
    // otherwise the epoch ends at the next normalisation, shortened until the watched set fits.
    const uint32_t v_next100 = (v0 / 100 + 1) * 100;
    uint32_t v_end = v_next100 + 1500;
    bool long_try = true;
    for (int attempt = 0; attempt < 5; ++attempt) {
        const uint32_t vl = v_end - 1;         // the epoch's last selection
        const float pc = pc_at(vl);
        const double sq = std::sqrt(vl + 1);
        double unwatched = -1e300;
        int nwatch = 0;
        bool watch_prior = false;
        bool ok = true;
        for (int j = 0; j < nother && ok; ++j) {
            const int i = other[j];
            const PuctNodeChild* c = cs + i;
            double base, expl;
            if (kind[i] == kUnexp) {
                base = prior_bound;
                expl = pc * c->policy_prob * sq / (c->traversals + 1 + 0.0);
            } else {
                base = S.base[i];
                expl = S.bcs[i] ? 0.0 : pc * c->policy_prob * sq / (c->traversals + 1 + 0.0);
            }
            const double u = spin_margin_up(base + expl);
            if (u < floor_adj) {
                unwatched = std::max(unwatched, u);
            } else if (nwatch == SpinEpoch::kMaxWatched) {
                ok = false;
            } else {
                spin.watched_flag[nwatch++] = (uint16_t)i;
                watch_prior = watch_prior || kind[i] == kUnexp;
            }
        }
        if (long_try) {
            long_try = false;
            if (!ok || nwatch != 0) {
                v_end = v_next100;
                continue;
            }
        }
        if (ok) {
            // wins and watched candidates in sortedChildrenSelect order (evaluator.cpp:242-263;
            // equal-score wins are equivalent under its comparator, so std::sort's permutation
            // decides)
            std::memset(watched, 0, n);
            for (int w = 0; w < nwatch; ++w) watched[spin.watched_flag[w]] = 1;
            const uint16_t* order = S.sortedOrder(n);
            // each candidate's position among the children the selection loop reaches (all but the
            // skipped bad-fallback ones): the index of its root-latch draw within a playout
            int k = 0, kw = 0, pos = 0;
            for (int j = 0; j < n; ++j) {
                const int i = order[j];
                if (kind[i] == kWinC) {
                    spin.cand[k] = (uint16_t)i;
                    spin.cand_pos[k] = (uint16_t)pos;
                    spin.cand_kind[k++] = SpinEpoch::kWin;
                    ++kw;
                } else if (watched[i]) {
                    spin.cand[k] = (uint16_t)i;
                    spin.cand_pos[k] = (uint16_t)pos;
                    spin.cand_kind[k++] = kind[i] == kUnexp ? SpinEpoch::kPrior : SpinEpoch::kScored;
                }
                if (kind[i] != kSkipC) ++pos;
            }
            // (a comparator that is not a strict weak ordering -- the reference's, with negative
            // scores next to unexpanded children -- may drop or repeat elements: ordinary path)
            if (kw != nw || k != nw + nwatch || pos != reach) return sd(kSdFailOrder), false;
            spin.ncand = k;
            spin.nvisited = nvis;
            spin.watch_prior = watch_prior;
            spin.regs_ok = regs_ok && !watch_prior && sm->roleCount() <= kMaxRoles;
            sd(kSdBuildOk);
            spin.win_score = win_score;
            spin.unwatched_bound = unwatched;
            spin.conv_false = conv_false;
            spin.root = node;
            spin.v_end = v_end;
            spin.reach = reach;
            spin.drift = 1.0;
            spin.valid = true;
            total_spin_epochs++;
            return true;
        }
        const uint32_t k = (v_end - v0) / 4;
        if (k == 0) break;
        v_end = v0 + k;
    }
    sd(kSdFailWatched);
    return false;
}

// Up to `limit` consecutive spin playouts (1 unless `multi`: playoutMain passes multi when none of
// its loop conditions can change over a run of spin playouts, see there); a run continues past the
// first playout only inside an epoch whose converged() is proved false.  Returns how many playouts
// ran (0: the next playout takes the ordinary path).  Each playout is spinPlayout's selection and
// backup() specialised to the path root -> finalised win: the same float / double operations in the
// same order, with no path vector and no per-playout loop-top bookkeeping.
int PuctEvaluator::spinRun(int limit, bool multi) {
    if (!spin_fast_enabled() || limit <= 0) return 0;
    if (spin.fail_next) {   // the playout after a run failed the fast path: ordinary path now
        spin.fail_next = false;
        spin.valid = false;
        return 0;
    }
    PuctNode* node = root;
    if (!spin.valid || spin.root != node || node->visits >= spin.v_end) {
        if (spin.root == node && node->visits < spin.retry_at) return sd(kSdRetryWait), 0;
        if (!spinBuild()) {
            spin.root = node;
            spin.retry_at = node->visits + 8;
            return 0;
        }
    }
    if (!multi || !spin.conv_false) limit = 1;
    const bool verify = verify_fastpath();
    if (spin.regs_ok && spin_fast_mode() == 1) {
        if (!verify) {
            const int r = spinRunRegs(limit);
            if (r >= 0) return r;
        } else {
            // verification: the register run, then the same run again from the same state through
            // the loop below (whose every playout is re-selected by the ordinary path); the two end
            // states must be identical
            const SpinSnapshot before = spinSnapshot();
            const int r = spinRunRegs(limit);
            if (r >= 0) {
                const SpinSnapshot regs = spinSnapshot();
                spinRestore(before);
                const int r2 = spinRunSlow(limit, true);
                const SpinSnapshot slow = spinSnapshot();
                if (r2 != r || !(regs == slow)) {
                    std::fprintf(stderr, "gz spin register-run mismatch (visits %u, playouts %d vs %d)\n", node->visits,
                                 r, r2);
                    std::abort();
                }
                count_verified();
                return r2;
            }
        }
    }
    return spinRunSlow(limit, verify);
}

// Everything a spin run may change (the root's allocation -- header, child entries, scores --, the
// candidates' node allocations, the epoch, the RNG and the counters), for GZ_VERIFY_FASTPATH.
PuctEvaluator::SpinSnapshot PuctEvaluator::spinSnapshot() const {
    SpinSnapshot s;
    auto add = [&s](const PuctNode* n) {
        const char* b = reinterpret_cast<const char*>(n);
        s.bytes.insert(s.bytes.end(), b, b + n->allocated_size);
    };
    add(root);
    // the child entries' debug scores are written by the verifying selection only (diagnostics)
    for (int i = 0; i < root->num_children; ++i) {
        PuctChildCold* c = reinterpret_cast<PuctChildCold*>(s.bytes.data() + sizeof(PuctNode) +
                                                            sizeof(PuctNodeChild) * root->num_children) + i;
        c->debug_node_score = 0.f;
        c->debug_puct_score = 0.f;
    }
    const PuctNodeChild* cs = root->children();
    for (int k = 0; k < spin.ncand; ++k) add(cs[spin.cand[k]].to_node);
    s.valid = spin.valid;
    s.fail_next = spin.fail_next;
    s.v_end = spin.v_end;
    s.drift = spin.drift;
    s.rng = rng;
    s.playouts_finals = stats.playouts_finals;
    s.num_tree_playouts = stats.num_tree_playouts;
    s.total_tree_playouts = total_tree_playouts;
    return s;
}

void PuctEvaluator::spinRestore(const SpinSnapshot& s) {
    size_t o = 0;
    auto put = [&s, &o](PuctNode* n) {
        const size_t sz = n->allocated_size;
        std::memcpy(reinterpret_cast<char*>(n), s.bytes.data() + o, sz);
        o += sz;
    };
    PuctNodeChild* cs = root->children();
    put(root);
    for (int k = 0; k < spin.ncand; ++k) put(cs[spin.cand[k]].to_node);
    spin.valid = s.valid;
    spin.fail_next = s.fail_next;
    spin.v_end = s.v_end;
    spin.drift = s.drift;
    rng = s.rng;
    stats.playouts_finals = s.playouts_finals;
    stats.num_tree_playouts = s.num_tree_playouts;
    total_tree_playouts = s.total_tree_playouts;
}

bool PuctEvaluator::SpinSnapshot::operator==(const SpinSnapshot& o) const {
    return bytes == o.bytes && valid == o.valid && fail_next == o.fail_next && v_end == o.v_end &&
           drift == o.drift && rng == o.rng &&
           playouts_finals == o.playouts_finals && num_tree_playouts == o.num_tree_playouts &&
           total_tree_playouts == o.total_tree_playouts;
}

// spinRun's playouts one at a time through the node structures (the reference's operations in its
// order); with `verify` every playout's choice is re-made by the ordinary selection.
int PuctEvaluator::spinRunSlow(int limit, bool verify) {
    PuctNode* node = root;
    const int lead = node->lead_role_index;
    const int role_count = sm->roleCount();
    PuctNodeChild* cs = node->children();
    const float limit_latch_root = 0.66;
    int done = 0;
    while (done < limit && node->visits < spin.v_end) {
        // a playout that cannot take the fast path ends the run; it is the ordinary path's, at once
        // when it is the run's first, else at the next call (after playoutMain's loop-top checks)
        auto fail = [&]() {
            if (done == 0) spin.valid = false;
            else spin.fail_next = true;
        };
        if (node->inflight_visits != 0 ||
            (!node->dirichlet_noise_set && conf->dirichlet_noise_pct >= 0 && node->getCurrentScore(lead) <= 0.95)) {
            fail();
            break;
        }

        // selectChild (evaluator.cpp:341-517) restricted to the wins and the watched candidates
        setPuctConstant(node, 0);
        const double sqrt_node_visits = std::sqrt(node->visits + 1);
        const bool latch = node->visits > 1000 && node->visits < 40000000;
        float prior_score = 0.f;
        if (spin.watch_prior) {
            // priorScore (evaluator.cpp:1195-1224): the top-visits child is a win; the policy sum of
            // the visited children accumulates in child order
            float total_policy_visited = 0.0;
            for (int k = 0; k < spin.nvisited; ++k) total_policy_visited += cs[spin.visited[k]].policy_prob;
            prior_score = spin.win_score;
            float fpu_reduction = conf->fpu_prior_discount_root;
            if (fpu_reduction > 0) {
                fpu_reduction *= std::sqrt(total_policy_visited);
                prior_score -= fpu_reduction;
            }
        }
        float best_score = -1;
        int best = -1;
        bool best_win = false;
        double best_exact = 0.0;
        // the root latch (evaluator.cpp:461-475): with the latch active every reached child draws
        // rng.get() in sorted order, and a child whose traversals exceed 0.66 v is left out of the
        // selection when its draw exceeds 0.1.  Only wins can be latched inside an epoch (spinBuild);
        // a latched win's draw is read at its position, the others are discarded unread.
        const Rng rng0 = rng;
        int drawn = 0;
        for (int k = 0; k < spin.ncand; ++k) {
            const int i = spin.cand[k];
            const uint8_t kind = spin.cand_kind[k];
            PuctNodeChild* c = cs + i;
            const PuctNode* cn = c->to_node;
            if (kind == SpinEpoch::kWin && latch && c->traversals > 16 &&
                c->traversals > node->visits * limit_latch_root) {
                if (drawn == 0) sd(kSdLatchDraws);
                rng.discard((uint64_t)(spin.cand_pos[k] - drawn));
                drawn = spin.cand_pos[k] + 1;
                if (rng.get() > 0.1) continue;
            }
            const int traversals = c->traversals + 1;
            const double inflight_visits = cn != nullptr ? cn->inflight_visits : 0;
            double exploration_score = node->puct_constant * c->policy_prob * sqrt_node_visits /
                                       (traversals + inflight_visits);
            double child_score = prior_score;
            if (cn != nullptr) {
                child_score = cn->getCurrentScore(lead);
                if (kind == SpinEpoch::kWin) child_score *= 1.0f + node->puct_constant;
                else if (cn->is_finalised) exploration_score = 0.0;
            }
            const double score = child_score + exploration_score;
            if (score > best_score) {   // the reference loop (evaluator.cpp:487-490), float best_score
                best = i;
                best_score = score;
                best_win = kind == SpinEpoch::kWin;
                best_exact = score;
            }
        }
        // a watched candidate wins (its playout descends: ordinary path), or the result is not
        // separated from the unwatched bound
        if (best < 0 || !best_win || !(spin.unwatched_bound < best_exact) ||
            !(spin.unwatched_bound <= (double)(float)best_exact)) {
            rng = rng0;
            fail();
            break;
        }
        PuctNodeChild* chosen = cs + best;
        if (latch) rng.discard((uint64_t)(spin.reach - drawn));   // the remaining draws (values unused)

        if (verify) {
            // the ordinary selection from the same RNG state must pick the same child
            const Rng after = rng;
            rng = rng0;
            Path tmp;
            PuctNodeChild* ref = selectChild(node, tmp);
            if (ref != chosen || !(rng == after)) {
                std::fprintf(stderr, "gz spin fast-path mismatch (visits %u)\n", node->visits);
                std::abort();
            }
            if (spin.conv_false && converged(conf->converged_visits)) {
                std::fprintf(stderr, "gz spin fast-path: converged() is true\n");
                std::abort();
            }
            count_verified();
        }

        // treePlayout (evaluator.cpp:658-720): root -> chosen (finalised terminal), then backup()
        // over that two-element path (backup_finalised is off in an epoch)
        PuctNode* leaf = chosen->to_node;
        node->inflight_visits++;
        node->syncParent();
        stats.playouts_finals++;
        float scores[kMaxRoles];
        for (int ii = 0; ii < role_count; ii++) scores[ii] = leaf->getCurrentScore(ii);
        // the leaf (finalised): its scores propagate unchanged
        leaf->visits++;
        if (leaf->inflight_visits > 0) leaf->inflight_visits--;
        leaf->syncParent();
        if (leaf->visits % 100 == 0) leaf->normaliseX();
        // the root (never finalised inside an epoch)
        for (int ii = 0; ii < role_count; ii++) {
            float visits = node->visits;
            if (visits > 100000) visits = 100000 + 0.1f * (visits - 100000);
            const float score = ((visits * node->getCurrentScore(ii) + scores[ii]) / (visits + 1.0f));
            node->setCurrentScore(ii, score);
        }
        node->visits++;
        if (node->inflight_visits > 0) node->inflight_visits--;
        node->syncParent();
        chosen->traversals++;
        if (node->visits > 23) {
            const float cur_score = node->getCurrentScore(node->lead_role_index);
            float apply, minimum;
            if (cur_score > 0.3 && cur_score < 0.7) {
                apply = 0.995;
                minimum = 0.02f;
            } else if (cur_score > 0.15 && cur_score < 0.85) {
                apply = 0.9975;
                minimum = 0.03f;
            } else {
                apply = 0.9975;
                minimum = 0.10f;
            }
            if (chosen->policy_prob > minimum) {
                chosen->policy_prob *= apply;
                chosen->policy_prob = std::max(minimum, chosen->policy_prob);
            }
        }
        if (node->visits % 100 == 0) {
            // normaliseX inside an epoch: the epoch expires when the rescaling drifts (spinBuild)
            float before[SpinEpoch::kMaxWins + SpinEpoch::kMaxWatched] = {};
            for (int k = 0; k < spin.ncand; ++k) before[k] = cs[spin.cand[k]].policy_prob;
            node->normaliseX();
            double dev = 0.0;
            for (int k = 0; k < spin.ncand; ++k)
                dev = std::max(dev, std::fabs((double)cs[spin.cand[k]].policy_prob / (double)before[k] - 1.0));
            spin.drift *= (double)cs[spin.cand[0]].policy_prob / (double)before[0];
            if (dev > kSpinDrift || std::fabs(spin.drift - 1.0) > 2 * kSpinDrift) spin.v_end = node->visits;
        }
        stats.num_tree_playouts++;
        total_tree_playouts++;
        ++done;
    }
    sd(kSdSlowPlayouts, done);
    return done;
}

// spinRun's playouts with the run's state in registers (the common epoch: no watched unexpanded
// child, every win a childless terminal node): the selection and backup of the loop above,
// operation for operation and in the same order, without the per-playout loads of the win nodes,
// mirror refreshes and child-entry round trips through memory.  The candidates' traversals and
// policy, the wins' visits and mirrors and the root's visits / scores / puct constant are written
// back once at the end of the run (nothing else reads them inside it); the root-latch discards are
// summed (Rng::discard only accumulates).  Steady-state engine probe (tools/engine_bench.cpp, one
// thread): ~4-5 % less time per leaf than the loop above, trajectories identical.
namespace {
struct SpinRegs {
    static constexpr int kC = 16;
    float P[kC];            // policy_prob
    uint32_t T[kC];         // traversals
    float BASE[kC];         // current score of the parent's lead role
    uint32_t LV[kC];        // the child node's visits
    bool WIN[kC], FIN[kC];
    float lsc[kC][kMaxRoles];
    float cur[kMaxRoles];   // the root's current scores
    int nc, lead, role_count;
    bool noise_check;
    float pc_root, pc;
    double ub;
    uint32_t v, v_end;
    uint64_t reach, discards = 0;
    uint32_t touched = 0;   // candidates chosen in this run (bit k)
    int done = 0;
    bool failed = false;
    PuctNode* node = nullptr;        // the root (normaliseX inside a run)
    const uint16_t* cand = nullptr;  // candidate k's child index
    double drift = 1.0;              // the epoch's product of normalisation factors
    bool expired = false;            // a normalisation drifted: the epoch ends after this playout
    int why = 0;                     // diagnostics (GZ_SPIN_STATS): 1 noise, 2 latch, 3 separation
    Rng* rng = nullptr;              // the evaluator's generator (root-latch draws read inside a run)
    uint16_t pos[kC];                // candidate k's position among the reached children (its draw)
};

// The root latch inside a register run (selectChild, evaluator.cpp:461-475): with the latch active
// each reached child draws rng.get() in sorted order and a child whose traversals exceed 0.66 v is
// left out of the selection when its draw exceeds 0.1.  Returns the mask of candidates left out of
// this playout; the pending discards (earlier playouts' unread draws) and the draws before each
// latched win are skipped, the playout's draws after the last latched one stay for the caller
// (reach - *drawn).  On a failed playout the caller restores the generator from `saved`.
struct LatchDraws {
    Rng saved;
    uint64_t saved_pending = 0;
    bool drew = false;
    int drawn = 0;
};
template <class TA>
inline uint32_t latch_skips(SpinRegs& x, const TA& T, int nc, uint32_t v, uint64_t& pending, LatchDraws& ld) {
    const float limit_latch_root = 0.66;
    uint32_t mask = 0;
    for (int k = 0; k < nc; ++k) {
        const uint32_t t = (uint32_t)T[k];
        if (!(x.WIN[k] && t > 16 && t > v * limit_latch_root)) continue;
        if (!ld.drew) {
            ld.saved = *x.rng;
            ld.saved_pending = pending;
            ld.drew = true;
            sd(kSdLatchDraws);
        }
        x.rng->discard(pending + (uint64_t)(x.pos[k] - ld.drawn));
        pending = 0;
        ld.drawn = x.pos[k] + 1;
        if (x.rng->get() > 0.1) mask |= 1u << k;
    }
    return mask;
}
inline void latch_undo(SpinRegs& x, uint64_t& pending, const LatchDraws& ld) {
    if (!ld.drew) return;
    *x.rng = ld.saved;
    pending = ld.saved_pending;
}

// normaliseX at the root inside a register run (backup, evaluator.cpp:650): the candidates'
// policies to the child entries, normalise, read them back; the epoch expires when the factor
// drifts (spinBuild's bounds assume the policies it read, within kSpinDrift)
inline void spin_normalise(SpinRegs& x, float* P, int nc) {
    PuctNodeChild* cs = x.node->children();
    float before[SpinRegs::kC];
    for (int k = 0; k < nc; ++k) {
        before[k] = P[k];
        cs[x.cand[k]].policy_prob = P[k];
    }
    x.node->normaliseX();
    double dev = 0.0;
    for (int k = 0; k < nc; ++k) {
        P[k] = cs[x.cand[k]].policy_prob;
        dev = std::max(dev, std::fabs((double)P[k] / (double)before[k] - 1.0));
    }
    x.drift *= (double)P[0] / (double)before[0];
    x.touched = (1u << nc) - 1;
    if (dev > kSpinDrift || std::fabs(x.drift - 1.0) > 2 * kSpinDrift) x.expired = true;
}

// backup()'s policy decay of the chosen child at the root (evaluator.cpp:605-625)
inline void decay_params(float cur_score, float* apply, float* minimum) {
    if (cur_score > 0.3 && cur_score < 0.7) {
        *apply = 0.995;
        *minimum = 0.02f;
    } else if (cur_score > 0.15 && cur_score < 0.85) {
        *apply = 0.9975;
        *minimum = 0.03f;
    } else {
        *apply = 0.9975;
        *minimum = 0.10f;
    }
}

// Every candidate a win with the same scores: NC candidates at compile time, so their state lives
// in registers.  (Deep in a spin -- root visits in the millions -- the wins' exploration terms differ
// by less than a float ulp of their scores and the choice is decided by the rounding of the
// reference's float `best_score`; the choice branches stay: predicted, they keep consecutive
// playouts overlapping, where selects measured ~1.7x slower by making the choice a data dependency.)
template <int NC, int R>
__attribute__((noinline)) void spin_wins(SpinRegs& x, int limit) {
    float P[NC];
    uint32_t T[NC], LV[NC];
    for (int k = 0; k < NC; ++k) { P[k] = x.P[k]; T[k] = x.T[k]; LV[k] = x.LV[k]; }
    const float win_base = x.BASE[0];
    float sc[R], cur[R];
    const int lead = x.lead;
    for (int ii = 0; ii < R; ii++) { sc[ii] = x.lsc[0][ii]; cur[ii] = x.cur[ii]; }
    // cur[lead] with the role unrolled (a runtime index would keep cur in memory)
    auto lead_score = [lead](const float* c) {
        float r = c[0];
        for (int ii = 1; ii < R; ii++) r = lead == ii ? c[ii] : r;
        return r;
    };
    const float pc_root = x.pc_root;
    const bool noise_check = x.noise_check;
    const double ub = x.ub;
    const uint32_t v_end = x.v_end;
    const uint64_t reach = x.reach;
    uint32_t v = x.v, touched = 0;
    float pc = x.pc;
    uint64_t discards = 0;
    int done = 0;
    bool failed = false;
    PuctLogCursor plog;
    // a win reaches the root latch only when its traversals exceed 0.66 v: over this run a win's
    // traversals grow by at most the run's length while v only grows, so when even that cannot
    // reach 0.66 v (with a margin far above the float rounding of both sides) no playout of the run
    // needs the check
    uint32_t tmax = 0;
    for (int k = 0; k < NC; ++k) tmax = std::max(tmax, T[k]);
    const uint32_t run_max = std::min<uint32_t>((uint32_t)std::max(limit, 0), v_end - v);
    const bool check_latch = !((double)tmax + run_max < 0.66 * (double)v * (1.0 - 1e-5));
    while (done < limit && v < v_end) {
        if (noise_check && lead_score(cur) <= 0.95) {
            failed = true;
            break;
        }
        pc = plog.at(v);
        pc += pc_root;
        const double sqrt_node_visits = sqrt_pos(v + 1);
        const bool latch = v > 1000 && v < 40000000;
        LatchDraws ld;
        const uint32_t skip = check_latch && latch ? latch_skips(x, T, NC, v, discards, ld) : 0u;
        double child_score = win_base;
        child_score *= 1.0f + pc;
        float best_score = -1;
        int best = -1;
        double best_exact = 0.0;
        for (int k = 0; k < NC; ++k) {
            if (skip >> k & 1) continue;
            const int traversals = T[k] + 1;
            const double inflight_visits = 0;
            const double exploration_score = pc * P[k] * sqrt_node_visits / (traversals + inflight_visits);
            const double score = child_score + exploration_score;
            if (score > best_score) {
                best = k;
                best_score = score;
                best_exact = score;
            }
        }
        if (best < 0 || !(ub < best_exact) || !(ub <= (double)(float)best_exact)) {
            latch_undo(x, discards, ld);
            failed = true;
            break;
        }
        discards += latch ? reach - ld.drawn : 0;
        touched |= 1u << best;
        for (int ii = 0; ii < R; ii++) {
            float visits = v;
            if (visits > 100000) visits = 100000 + 0.1f * (visits - 100000);
            cur[ii] = ((visits * cur[ii] + sc[ii]) / (visits + 1.0f));
        }
        v++;
        // the chosen candidate's updates through unrolled per-candidate predicates (compile-time
        // indices keep the arrays in registers; an update at index `best` would put them in memory)
        float apply = 1.0f, minimum = 0.0f;
        const bool dec = v > 23;
        if (dec) decay_params(lead_score(cur), &apply, &minimum);
        for (int k = 0; k < NC; ++k) {
            const bool ch = k == best;
            LV[k] += ch;
            T[k] += ch;
            const float p = P[k];
            float pn = p * apply;
            pn = std::max(minimum, pn);
            P[k] = ch && dec && p > minimum ? pn : p;
        }
        ++done;
        if (v % 100 == 0) {
            spin_normalise(x, P, NC);
            if (x.expired) break;
        }
    }
    for (int k = 0; k < NC; ++k) { x.P[k] = P[k]; x.T[k] = T[k]; x.LV[k] = LV[k]; }
    for (int ii = 0; ii < R; ii++) x.cur[ii] = cur[ii];
    x.v = v;
    x.pc = pc;
    x.discards += discards;
    x.touched |= touched;
    x.done += done;
    x.failed = failed;
}

// spin_wins for two roles and up to four all-win candidates, with the per-candidate arithmetic in
// AVX2 lanes: the candidates' exploration terms are one packed float multiply (pc * P, float as in the
// reference), one packed double multiply and ONE packed double division (vdivpd) instead of NC scalar
// divisions, and the state stays in vector registers.  Lane k computes exactly the scalar expression
// of candidate k (IEEE packed arithmetic, no contraction), so the choice is the same.  The root's
// current scores are updated speculatively: deep in a spin cur = (v cur + s) / (v + 1) rounds back to
// cur, so the update is computed from the held value and compared (bitwise) instead of chained through
// every playout's divisions -- a changed value is taken as usual.
template <int NC>
__attribute__((noinline, target("avx2"))) void spin_wins_v(SpinRegs& x, int limit) {
    static_assert(NC >= 2 && NC <= 4, "lanes");
    alignas(32) float Pa[4] = {0.f, 0.f, 0.f, 0.f};
    alignas(16) int32_t Ta[4] = {0, 0, 0, 0};
    for (int k = 0; k < NC; ++k) { Pa[k] = x.P[k]; Ta[k] = (int32_t)x.T[k]; }
    uint32_t LV[NC], T0[NC];
    for (int k = 0; k < NC; ++k) { LV[k] = x.LV[k]; T0[k] = x.T[k]; }
    __m128 Pv = _mm_load_ps(Pa);
    __m128i Tv = _mm_load_si128((const __m128i*)Ta);
    const __m128i lane_id = _mm_set_epi32(3, 2, 1, 0);
    const __m128i one_i = _mm_set1_epi32(1);
    const float win_base = x.BASE[0];
    const float sc0 = x.lsc[0][0], sc1 = x.lsc[0][1];
    float cur0 = x.cur[0], cur1 = x.cur[1];
    const int lead = x.lead;
    const float pc_root = x.pc_root;
    const bool noise_check = x.noise_check;
    const double ub = x.ub;
    const uint32_t v_end = x.v_end;
    const uint64_t reach = x.reach;
    uint32_t v = x.v, touched = 0;
    float pc = x.pc;
    uint64_t discards = 0;
    int done = 0;
    bool failed = false;
    PuctLogCursor plog;
    uint32_t tmax = 0;
    for (int k = 0; k < NC; ++k) tmax = std::max(tmax, x.T[k]);
    const uint32_t run_max = std::min<uint32_t>((uint32_t)std::max(limit, 0), v_end - v);
    const bool check_latch = !((double)tmax + run_max < 0.66 * (double)v * (1.0 - 1e-5));
    alignas(32) double sa[4];
    while (done < limit && v < v_end) {
        const float lead_cur = lead == 0 ? cur0 : cur1;
        if (noise_check && lead_cur <= 0.95) {
            failed = true;
            break;
        }
        pc = plog.at(v);
        pc += pc_root;
        const double sqrt_node_visits = sqrt_pos(v + 1);
        const bool latch = v > 1000 && v < 40000000;
        LatchDraws ld;
        uint32_t skip = 0;
        if (check_latch && latch) {
            _mm_store_si128((__m128i*)Ta, Tv);
            skip = latch_skips(x, Ta, NC, v, discards, ld);
        }
        double child_score = win_base;
        child_score *= 1.0f + pc;
        // exploration_score = pc * P[k] * sqrt_node_visits / (traversals + 0.0), traversals = T[k] + 1
        const __m128 pcP = _mm_mul_ps(_mm_set1_ps(pc), Pv);
        const __m256d num = _mm256_mul_pd(_mm256_cvtps_pd(pcP), _mm256_set1_pd(sqrt_node_visits));
        const __m256d den = _mm256_add_pd(_mm256_cvtepi32_pd(_mm_add_epi32(Tv, one_i)), _mm256_setzero_pd());
        const __m256d score = _mm256_add_pd(_mm256_set1_pd(child_score), _mm256_div_pd(num, den));
        _mm256_store_pd(sa, score);
        float best_score = -1;
        int best = -1;
        double best_exact = 0.0;
        for (int k = 0; k < NC; ++k) {
            if (!(skip >> k & 1) && sa[k] > best_score) {
                best = k;
                best_score = sa[k];
                best_exact = sa[k];
            }
        }
        if (best < 0 || !(ub < best_exact) || !(ub <= (double)(float)best_exact)) {
            latch_undo(x, discards, ld);
            failed = true;
            break;
        }
        discards += latch ? reach - ld.drawn : 0;
        touched |= 1u << best;
        {
            float visits = v;
            if (visits > 100000) visits = 100000 + 0.1f * (visits - 100000);
            const float n0 = ((visits * cur0 + sc0) / (visits + 1.0f));
            const float n1 = ((visits * cur1 + sc1) / (visits + 1.0f));
            // (bitwise: the update is taken whenever it changes a bit)
            if (__builtin_expect(__builtin_bit_cast(uint32_t, n0) != __builtin_bit_cast(uint32_t, cur0), 0)) cur0 = n0;
            if (__builtin_expect(__builtin_bit_cast(uint32_t, n1) != __builtin_bit_cast(uint32_t, cur1), 0)) cur1 = n1;
        }
        v++;
        const __m128i sel = _mm_cmpeq_epi32(lane_id, _mm_set1_epi32(best));
        Tv = _mm_sub_epi32(Tv, sel);                     // T[best] += 1 (sel lanes are -1)
        if (v > 23) {
            float apply = 1.0f, minimum = 0.0f;
            decay_params(lead == 0 ? cur0 : cur1, &apply, &minimum);
            // P[best] = max(minimum, P[best] * apply) when P[best] > minimum (std::max(a, b): b if a < b)
            const __m128 mn = _mm_set1_ps(minimum);
            const __m128 pn = _mm_mul_ps(Pv, _mm_set1_ps(apply));
            const __m128 clamped = _mm_blendv_ps(mn, pn, _mm_cmplt_ps(mn, pn));
            const __m128 upd = _mm_and_ps(_mm_castsi128_ps(sel), _mm_cmpgt_ps(Pv, mn));
            Pv = _mm_blendv_ps(Pv, clamped, upd);
        }
        ++done;
        if (v % 100 == 0) {
            _mm_store_ps(Pa, Pv);
            spin_normalise(x, Pa, NC);
            Pv = _mm_load_ps(Pa);
            if (x.expired) break;
        }
    }
    _mm_store_ps(Pa, Pv);
    _mm_store_si128((__m128i*)Ta, Tv);
    for (int k = 0; k < NC; ++k) {
        x.P[k] = Pa[k];
        x.T[k] = (uint32_t)Ta[k];
        x.LV[k] = LV[k] + ((uint32_t)Ta[k] - T0[k]);   // the win's visits rise with its traversals
    }
    x.cur[0] = cur0;
    x.cur[1] = cur1;
    x.v = v;
    x.pc = pc;
    x.discards += discards;
    x.touched |= touched;
    x.done += done;
    x.failed = failed;
}

// spin_wins_v in blocks of up to 8 playouts (GZ_SPIN_VEC=2).  Everything a playout computes that
// does not depend on which candidate the earlier playouts chose is computed for the whole block
// with packed instructions before the block's selections run: the puct constants (table lookups),
// sqrt(visits + 1) (two packed square roots instead of eight), and the root's current scores -- deep
// in a spin cur = (v cur + s) / (v + 1) rounds back to cur, so one packed division per role checks
// eight playouts' updates at once; the block ends at the first playout whose update changes a bit
// (taken there, exactly as the per-playout loop takes it), at the next root normalisation and at the
// run's limits.  With cur fixed over the block, the noise check and the policy decay's parameters are
// the block's too.  What stays per playout is the choice itself: one packed float multiply, one
// packed double multiply and one packed double division for the NC candidates, and the float-rounded
// comparisons in candidate order.  Every value is the scalar loop's (IEEE packed arithmetic, no
// contraction): the choice and the state are the same bit for bit.
template <int NC>
__attribute__((noinline, target("avx2"))) void spin_wins_b(SpinRegs& x, int limit) {
    static_assert(NC >= 2 && NC <= 4, "lanes");
    constexpr int kB = 8;
    alignas(32) float Pa[4] = {0.f, 0.f, 0.f, 0.f};
    alignas(16) int32_t Ta[4] = {0, 0, 0, 0};
    for (int k = 0; k < NC; ++k) { Pa[k] = x.P[k]; Ta[k] = (int32_t)x.T[k]; }
    uint32_t LV[NC], T0[NC];
    for (int k = 0; k < NC; ++k) { LV[k] = x.LV[k]; T0[k] = x.T[k]; }
    __m128 Pv = _mm_load_ps(Pa);
    __m128i Tv = _mm_load_si128((const __m128i*)Ta);
    const __m128i lane_id = _mm_set_epi32(3, 2, 1, 0);
    const __m128i one_i = _mm_set1_epi32(1);
    const float win_base = x.BASE[0];
    const float sc0 = x.lsc[0][0], sc1 = x.lsc[0][1];
    float cur0 = x.cur[0], cur1 = x.cur[1];
    const int lead = x.lead;
    const float pc_root = x.pc_root;
    const bool noise_check = x.noise_check;
    const double ub = x.ub;
    const uint32_t v_end = x.v_end;
    const uint64_t reach = x.reach;
    uint32_t v = x.v, touched = 0;
    float pc = x.pc;
    uint64_t discards = 0;
    int done = 0;
    bool failed = false;
    PuctLogCursor plog;
    uint32_t tmax = 0;
    for (int k = 0; k < NC; ++k) tmax = std::max(tmax, x.T[k]);
    const uint32_t run_max = std::min<uint32_t>((uint32_t)std::max(limit, 0), v_end - v);
    const bool check_latch = !((double)tmax + run_max < 0.66 * (double)v * (1.0 - 1e-5));
    alignas(32) double sa[4];
    alignas(32) float pcs[kB];
    alignas(32) double sqs[kB];
    alignas(32) float n0s[kB], n1s[kB];
    const __m256i jv = _mm256_set_epi32(7, 6, 5, 4, 3, 2, 1, 0);
    while (done < limit && v < v_end) {
        if (noise_check && (lead == 0 ? cur0 : cur1) <= 0.95) {
            failed = true; x.why = 1;
            break;
        }
        // block length: the run's limits and the next root normalisation (after the playout that
        // brings v to a multiple of 100)
        int L = kB;
        L = std::min<int>(L, limit - done);
        L = std::min<int>(L, (int)(v_end - v));
        L = std::min<int>(L, 100 - (int)(v % 100));
        // the block's puct constants and square roots (independent of the choices)
        for (int j = 0; j < L; ++j) {
            float p = plog.at(v + j);
            p += pc_root;
            pcs[j] = p;
        }
        {
            const __m256i vj1 = _mm256_add_epi32(_mm256_set1_epi32((int)v + 1), jv);   // v + j + 1 (< 2^31)
            _mm256_store_pd(sqs, _mm256_sqrt_pd(_mm256_cvtepi32_pd(_mm256_castsi256_si128(vj1))));
            _mm256_store_pd(sqs + 4, _mm256_sqrt_pd(_mm256_cvtepi32_pd(_mm256_extracti128_si256(vj1, 1))));
        }
        // the root's current-score updates of the block's playouts with cur held: visits = v + j
        // (> 100000: 100000 + 0.1 (visits - 100000)), n = (visits cur + s) / (visits + 1)
        int jchg = L;   // first playout whose update changes cur (it is taken there)
        {
            __m256 vis = _mm256_cvtepi32_ps(_mm256_add_epi32(_mm256_set1_epi32((int)v), jv));
            const __m256 big = _mm256_set1_ps(100000.f);
            const __m256 adj = _mm256_add_ps(big, _mm256_mul_ps(_mm256_set1_ps(0.1f), _mm256_sub_ps(vis, big)));
            vis = _mm256_blendv_ps(vis, adj, _mm256_cmp_ps(vis, big, _CMP_GT_OQ));
            const __m256 den = _mm256_add_ps(vis, _mm256_set1_ps(1.0f));
            const __m256 n0 = _mm256_div_ps(_mm256_add_ps(_mm256_mul_ps(vis, _mm256_set1_ps(cur0)), _mm256_set1_ps(sc0)), den);
            const __m256 n1 = _mm256_div_ps(_mm256_add_ps(_mm256_mul_ps(vis, _mm256_set1_ps(cur1)), _mm256_set1_ps(sc1)), den);
            // bitwise comparison (as the per-playout loop's)
            const __m256i c0 = _mm256_cmpeq_epi32(_mm256_castps_si256(n0), _mm256_set1_epi32(__builtin_bit_cast(int32_t, cur0)));
            const __m256i c1 = _mm256_cmpeq_epi32(_mm256_castps_si256(n1), _mm256_set1_epi32(__builtin_bit_cast(int32_t, cur1)));
            const uint32_t diff = ~(uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_and_si256(c0, c1))) & ((1u << L) - 1);
            if (diff) {
                jchg = __builtin_ctz(diff);
                _mm256_store_ps(n0s, n0);
                _mm256_store_ps(n1s, n1);
            }
        }
        const int Lb = jchg < L ? jchg + 1 : L;
        // the policy decay's parameters with cur held (and, for the last playout, with its update)
        float apply = 1.0f, minimum = 0.0f;
        decay_params(lead == 0 ? cur0 : cur1, &apply, &minimum);
        for (int j = 0; j < Lb; ++j) {
            const uint32_t vj = v + j;
            pc = pcs[j];
            const bool latch = vj > 1000 && vj < 40000000;
            LatchDraws ld;
            uint32_t skip = 0;
            if (check_latch && latch) {
                _mm_store_si128((__m128i*)Ta, Tv);
                skip = latch_skips(x, Ta, NC, vj, discards, ld);
            }
            double child_score = win_base;
            child_score *= 1.0f + pc;
            const __m128 pcP = _mm_mul_ps(_mm_set1_ps(pc), Pv);
            const __m256d num = _mm256_mul_pd(_mm256_cvtps_pd(pcP), _mm256_set1_pd(sqs[j]));
            const __m256d den = _mm256_add_pd(_mm256_cvtepi32_pd(_mm_add_epi32(Tv, one_i)), _mm256_setzero_pd());
            const __m256d score = _mm256_add_pd(_mm256_set1_pd(child_score), _mm256_div_pd(num, den));
            _mm256_store_pd(sa, score);
            float best_score = -1;
            int best = -1;
            double best_exact = 0.0;
            for (int k = 0; k < NC; ++k) {
                if (!(skip >> k & 1) && sa[k] > best_score) {
                    best = k;
                    best_score = sa[k];
                    best_exact = sa[k];
                }
            }
            if (best < 0 || !(ub < best_exact) || !(ub <= (double)(float)best_exact)) {
                latch_undo(x, discards, ld);
                failed = true; x.why = 3;
                break;
            }
            discards += latch ? reach - ld.drawn : 0;
            touched |= 1u << best;
            if (j == jchg) {   // this playout's update changes cur: taken, and its decay reads it
                cur0 = n0s[j];
                cur1 = n1s[j];
                decay_params(lead == 0 ? cur0 : cur1, &apply, &minimum);
            }
            const __m128i sel = _mm_cmpeq_epi32(lane_id, _mm_set1_epi32(best));
            Tv = _mm_sub_epi32(Tv, sel);
            if (vj + 1 > 23) {
                const __m128 mn = _mm_set1_ps(minimum);
                const __m128 pn = _mm_mul_ps(Pv, _mm_set1_ps(apply));
                const __m128 clamped = _mm_blendv_ps(mn, pn, _mm_cmplt_ps(mn, pn));
                const __m128 upd = _mm_and_ps(_mm_castsi128_ps(sel), _mm_cmpgt_ps(Pv, mn));
                Pv = _mm_blendv_ps(Pv, clamped, upd);
            }
            ++done;
        }
        v = x.v + done;   // (x.v: the run's first visit count)
        if (failed) break;
        if (v % 100 == 0) {
            _mm_store_ps(Pa, Pv);
            spin_normalise(x, Pa, NC);
            Pv = _mm_load_ps(Pa);
            if (x.expired) break;
        }
    }
    _mm_store_ps(Pa, Pv);
    _mm_store_si128((__m128i*)Ta, Tv);
    for (int k = 0; k < NC; ++k) {
        x.P[k] = Pa[k];
        x.T[k] = (uint32_t)Ta[k];
        x.LV[k] = LV[k] + ((uint32_t)Ta[k] - T0[k]);   // the win's visits rise with its traversals
    }
    x.cur[0] = cur0;
    x.cur[1] = cur1;
    x.v = v;
    x.pc = pc;
    x.discards += discards;
    x.touched |= touched;
    x.done += done;
    x.failed = failed;
}

// any candidate mix (wins and watched scored children)
void spin_mixed(SpinRegs& x, int limit) {
    const int nc = x.nc, lead = x.lead, role_count = x.role_count;
    while (x.done < limit && x.v < x.v_end) {
        if (x.noise_check && x.cur[lead] <= 0.95) {
            x.failed = true; x.why = 1;
            break;
        }
        const uint32_t v = x.v;
        float pc = puct_log(v);
        pc += x.pc_root;
        x.pc = pc;
        const double sqrt_node_visits = std::sqrt(v + 1);
        const bool latch = v > 1000 && v < 40000000;
        float best_score = -1;
        int best = -1;
        double best_exact = 0.0;
        LatchDraws ld;
        const uint32_t skip = latch ? latch_skips(x, x.T, nc, v, x.discards, ld) : 0u;
        for (int k = 0; k < nc; ++k) {
            if (skip >> k & 1) continue;
            const int traversals = x.T[k] + 1;
            const double inflight_visits = 0;
            double exploration_score = pc * x.P[k] * sqrt_node_visits / (traversals + inflight_visits);
            double child_score = x.BASE[k];
            if (x.WIN[k]) child_score *= 1.0f + pc;
            else if (x.FIN[k]) exploration_score = 0.0;
            const double score = child_score + exploration_score;
            if (score > best_score) {
                best = k;
                best_score = score;
                best_exact = score;
            }
        }
        if (best < 0 || !x.WIN[best] || !(x.ub < best_exact) || !(x.ub <= (double)(float)best_exact)) {
            latch_undo(x, x.discards, ld);
            x.failed = true; x.why = 3;
            break;
        }
        if (latch) x.discards += x.reach - ld.drawn;
        x.touched |= 1u << best;
        x.LV[best]++;
        for (int ii = 0; ii < role_count; ii++) {
            float visits = v;
            if (visits > 100000) visits = 100000 + 0.1f * (visits - 100000);
            x.cur[ii] = ((visits * x.cur[ii] + x.lsc[best][ii]) / (visits + 1.0f));
        }
        x.v = v + 1;
        x.T[best]++;
        if (x.v > 23) {
            float apply, minimum;
            decay_params(x.cur[lead], &apply, &minimum);
            if (x.P[best] > minimum) {
                x.P[best] *= apply;
                x.P[best] = std::max(minimum, x.P[best]);
            }
        }
        ++x.done;
        if (x.v % 100 == 0) {
            spin_normalise(x, x.P, nc);
            if (x.expired) break;
        }
    }
}
}  // namespace

// Returns -1 when a precondition fails at entry (spinRun's loop then runs), else the playouts run
// (0: the next playout takes the ordinary path, with spinRun's fail / fail_next convention).
int PuctEvaluator::spinRunRegs(int limit) {
    PuctNode* node = root;
    PuctNodeChild* cs = node->children();
    const int nc = spin.ncand;
    if (node->inflight_visits != 0 || nc > SpinRegs::kC) return -1;
    SpinRegs x;
    x.nc = nc;
    x.lead = node->lead_role_index;
    x.role_count = sm->roleCount();
    bool all_win = true;
    for (int k = 0; k < nc; ++k) {
        const PuctNodeChild* c = cs + spin.cand[k];
        const PuctNode* cn = c->to_node;
        if (cn == nullptr || cn->inflight_visits != 0) return -1;
        x.P[k] = c->policy_prob;
        x.T[k] = c->traversals;
        x.BASE[k] = cn->getCurrentScore(x.lead);
        x.LV[k] = cn->visits;
        x.WIN[k] = spin.cand_kind[k] == SpinEpoch::kWin;
        x.FIN[k] = cn->is_finalised;
        if (x.WIN[k] && cn->num_children != 0) return -1;
        for (int ii = 0; ii < x.role_count; ii++) {
            x.lsc[k][ii] = cn->getCurrentScore(ii);
            all_win = all_win && x.lsc[k][ii] == x.lsc[0][ii];
        }
        all_win = all_win && x.WIN[k];
    }
    for (int ii = 0; ii < x.role_count; ii++) x.cur[ii] = node->getCurrentScore(ii);
    x.noise_check = !node->dirichlet_noise_set && conf->dirichlet_noise_pct >= 0;
    x.pc_root = conf->puct_constant_root;
    x.pc = node->puct_constant;
    x.ub = spin.unwatched_bound;
    x.v = node->visits;
    x.v_end = spin.v_end;
    x.reach = (uint64_t)spin.reach;
    x.node = node;
    x.cand = spin.cand;
    x.drift = spin.drift;
    x.rng = &rng;
    for (int k = 0; k < nc; ++k) x.pos[k] = spin.cand_pos[k];
    // Register loops for all-win epochs: GZ_SPIN_VEC=2 (default) the AVX2 loop in blocks of eight
    // playouts, =1 the AVX2 loop per playout, =0 the scalar loop (all compute the same playouts).
    // On the GPU box's EPYC 9575F the AVX2 loops ran +4.7 % leaf-evals/s over the scalar one in the
    // bench's aged window (profiles/r05h_bench_*.log), the block form even with the per-playout one
    // (profiles/r05i_*; run-to-run spread ~4 %); it does a third of the divider work per playout.
    static const int vec = [] {
        const char* e = std::getenv("GZ_SPIN_VEC");
        return e != nullptr ? std::atoi(e) : 2;
    }();
    if (all_win && x.role_count == 2 && nc >= 2 && nc <= 4 && vec == 2) {
        if (nc == 2) spin_wins_b<2>(x, limit);
        else if (nc == 3) spin_wins_b<3>(x, limit);
        else spin_wins_b<4>(x, limit);
    } else if (all_win && x.role_count == 2 && nc == 2) vec ? spin_wins_v<2>(x, limit) : spin_wins<2, 2>(x, limit);
    else if (all_win && x.role_count == 2 && nc == 3) vec ? spin_wins_v<3>(x, limit) : spin_wins<3, 2>(x, limit);
    else if (all_win && x.role_count == 2 && nc == 4) vec ? spin_wins_v<4>(x, limit) : spin_wins<4, 2>(x, limit);
    else spin_mixed(x, limit);
    const int done = x.done;
    // write back (a selection that failed still ran setPuctConstant)
    if (done > 0 || x.failed) node->puct_constant = x.pc;
    for (int k = 0; k < nc; ++k) {
        if (!(x.touched & (1u << k))) continue;
        PuctNodeChild* c = cs + spin.cand[k];
        c->policy_prob = x.P[k];
        c->traversals = x.T[k];
        c->to_node->visits = x.LV[k];
        c->to_node->syncParent();
    }
    spin.drift = x.drift;
    if (x.expired) spin.v_end = x.v;   // the next call rebuilds the epoch
    if (done > 0) {
        node->visits = x.v;
        for (int ii = 0; ii < x.role_count; ii++) node->setCurrentScore(ii, x.cur[ii]);
        node->syncParent();
        stats.playouts_finals += done;
        stats.num_tree_playouts += done;
        total_tree_playouts += done;
        rng.discard(x.discards);
    }
    if (x.failed) {
        if (done == 0) spin.valid = false;
        else spin.fail_next = true;
    }
    sd(kSdRegsPlayouts, done);
    if (__builtin_expect(g_spin_stats.on, 0)) {
        sd(kSdRegRuns);
        if (x.failed) sd(x.why == 1 ? kSdRegFailNoise : x.why == 2 ? kSdRegFailLatch : kSdRegFailSep);
        if (x.expired) sd(kSdRegExpired);
    }
    return done;
}

// evaluator.cpp:722-742
void PuctEvaluator::playoutWorker(int) {
    while (do_playouts) {
        if (stats.num_tree_playouts % 10000 == 0) scheduler->yield();
        if (root->is_finalised) break;
        Path path;
        const int depth = treePlayout(root, path);
        stats.playouts_max_depth = std::max(depth, stats.playouts_max_depth);
        stats.playouts_total_depth += depth;
    }
}

// evaluator.cpp:744-886 (verbose reporting omitted)
void PuctEvaluator::playoutMain(int max_evaluations, double end_time) {
    const double start_time = get_time();
    const bool use_think_time = conf->think_time > 0;
    auto elapsed = [start_time](double t) { return get_time() > (start_time + t); };

    const int max_non_converged_evaluations = max_evaluations * conf->evaluation_multiplier_to_convergence;
    const int max_tree_playouts = 4 * max_non_converged_evaluations;

    Path path;
    int evals_seen = stats.num_evaluations, quiet_playouts = 0;   // spin_yield_playouts (config.h)
    spin.fail_next = false;   // a failure seen past the end of the last call is re-evaluated
    while (true) {
        const int our_role_index = root->lead_role_index;
        // converged() is pure (no RNG, no writes); the reference evaluates it every iteration, but
        // without think time its value can only matter once tree playouts exceed max_tree_playouts
        // or evaluations exceed either evaluation limit, so it is evaluated lazily (same decisions).
        const bool need_converged = use_think_time || stats.num_tree_playouts > max_tree_playouts ||
                                    stats.num_evaluations > max_evaluations ||
                                    stats.num_evaluations > max_non_converged_evaluations;
        // inside a spin epoch converged() may be provably false (spinBuild)
        const bool spin_epoch = spin.valid && spin.conv_false && spin.root == root && root->visits < spin.v_end;
        const bool is_converged = need_converged && !spin_epoch ? converged(conf->converged_visits) : false;

        // (diagnostics: GZ_SPIN_STATS counts the exits and the NN-free playouts of their moves)
        auto exit_stat = [&](SpinStat e, SpinStat f) {
            if (__builtin_expect(!g_spin_stats.on, 1)) return;
            sd(e);
            if (f != kSdCount) sd(f, stats.num_tree_playouts - stats.num_evaluations);
        };
        if (end_time > 0 && get_time() > end_time) { exit_stat(kSdExitOther, kSdCount); break; }
        if (root->is_finalised && stats.num_tree_playouts > 100) { exit_stat(kSdExitFinal, kSdCount); break; }
        if (is_converged && stats.num_tree_playouts > max_tree_playouts) {
            exit_stat(kSdExitConvPlayouts, kSdFreeAtConvPlayouts);
            break;
        }
        if (number_of_nodes > 50000000) { exit_stat(kSdExitOther, kSdCount); break; }
        if (is_converged && stats.num_evaluations > max_evaluations) {
            exit_stat(kSdExitConvEvals, kSdFreeAtConvEvals);
            break;
        }
        if (!is_converged && stats.num_evaluations > max_non_converged_evaluations) {
            exit_stat(kSdExitNonConvEvals, kSdFreeAtNonConvEvals);
            break;
        }
        if (use_think_time) {
            if (is_converged && elapsed(conf->think_time)) break;
            if (!is_converged && elapsed(conf->think_time * conf->evaluation_multiplier_to_convergence)) break;
            if (elapsed(120.0) && is_converged) {
                const PuctNodeChild* best = chooseTopVisits(root);
                if (best->to_node->getCurrentScore(our_role_index) > 0.975 ||
                    best->to_node->getCurrentScore(our_role_index) < 0.025)
                    break;
            }
        }

        // A run of spin playouts stands for that many iterations of this loop when none of the
        // checks above can change within it: no think time or end time, the non-converged
        // evaluation limit not reached (evaluations and node counts do not change in a spin
        // playout), converged() proved false (spinRun), and the run ends at the next spin yield.
        const bool multi = !use_think_time && end_time <= 0 && !root->is_finalised &&
                           !(stats.num_evaluations > max_non_converged_evaluations) && number_of_nodes <= 50000000;
        int limit = 1 << 20;
        if (conf->spin_yield_playouts > 0) limit = conf->spin_yield_playouts - quiet_playouts;
        int depth = 2;
        const uint64_t c0 = __builtin_expect(g_spin_stats.on, 0) ? __rdtsc() : 0;
        int ran = spinRun(limit, multi);
        if (__builtin_expect(g_spin_stats.on, 0) && ran > 0) sd(kSdCycSpin, (long)(__rdtsc() - c0));
        if (ran == 0) {
            spin.valid = false;
            path.clear();
            const int ev0 = stats.num_evaluations;
            const uint64_t c1 = __builtin_expect(g_spin_stats.on, 0) ? __rdtsc() : 0;
            depth = treePlayout(root, path);
            if (__builtin_expect(g_spin_stats.on, 0))
                sd(stats.num_evaluations == ev0 ? kSdCycFree : kSdCycEval, (long)(__rdtsc() - c1));
            ran = 1;
            sd(kSdOrdinaryPlayouts);
            if (__builtin_expect(g_spin_stats.on, 0) && stats.num_evaluations == ev0 &&
                stats.num_tree_playouts - stats.num_evaluations == spin_dump_at()) {
                // diagnostics (GZ_SPIN_DUMP=<n>): the root and the last playout's path once a move
                // has run n NN-free playouts (at most 6 dumps per process)
                static std::atomic<int> dumps{0};
                if (dumps.fetch_add(1) < 6) {
                    const int lead = root->lead_role_index;
                    std::fprintf(stderr, "gz spin dump: depth %d root visits %u lead %d score %.6f evals %d playouts %d\n",
                                 root->game_depth, root->visits, lead, root->getCurrentScore(lead < 0 ? 0 : lead),
                                 stats.num_evaluations, stats.num_tree_playouts);
                    for (int i = 0; i < root->num_children; ++i) {
                        const PuctNodeChild* c = root->getNodeChild(0, i);
                        const PuctNode* cn = c->to_node;
                        std::fprintf(stderr, "  child %2d trav %9u pol %.4f", i, c->traversals, c->policy_prob);
                        if (cn)
                            std::fprintf(stderr, " visits %9u score %.6f fin %d nch %d term %d\n", cn->visits,
                                         cn->getCurrentScore(lead), (int)cn->is_finalised, cn->num_children,
                                         (int)cn->isTerminal());
                        else
                            std::fprintf(stderr, " unexpanded\n");
                    }
                    for (size_t k = 0; k < path.size(); ++k) {
                        const PuctNode* n = path[k].node;
                        const int l = n->lead_role_index;
                        int ci = -1;
                        for (int i = 0; i < n->num_children && path[k].choice; ++i)
                            if (n->getNodeChild(0, i) == path[k].choice) ci = i;
                        std::fprintf(stderr, "  path %zu: lead %d visits %u score(lead) %.6f fin %d nch %d -> child %d\n", k, l,
                                     n->visits, n->getCurrentScore(l < 0 ? 0 : l), (int)n->is_finalised, n->num_children, ci);
                    }
                }
            }
            if (__builtin_expect(g_spin_stats.on, 0) && stats.num_evaluations == ev0) {
                int nw = 0;
                for (int i = 0; i < root->num_children; ++i) {
                    const PuctNode* cn = root->getNodeChild(0, i)->to_node;
                    if (cn != nullptr && cn->is_finalised && cn->getCurrentScore(root->lead_role_index) > 0.99) ++nw;
                }
                sd(nw == 0 ? kSdFree0 : nw == 1 ? kSdFree1 : kSdFree2);
                sd(depth <= 2 ? kSdFreeD2 : depth == 3 ? kSdFreeD3 : depth == 4 ? kSdFreeD4 : depth == 5 ? kSdFreeD5 : kSdFreeD6);
                if (depth == 3 && path[2].node->is_finalised && path[1].node->lead_role_index >= 0 &&
                    path[2].node->getCurrentScore(path[1].node->lead_role_index) > 0.99)
                    sd(kSdFreeX1Win);
                if (convergedExact(conf->converged_visits)) sd(kSdFreeConv);
                bool line = true;
                for (size_t k = 1; k + 1 < path.size() && line; ++k) {
                    const PuctNode* pn = path[k].node;
                    const PuctNodeChild* pc = path[k].choice;
                    line = pn->num_children == 1 ||
                           (pc && pc->to_node && pc->to_node->is_finalised && pn->lead_role_index >= 0 &&
                            pc->to_node->getCurrentScore(pn->lead_role_index) > 0.99);
                }
                if (line) sd(kSdFreeLine);
            }
        }
        stats.playouts_max_depth = std::max(depth, stats.playouts_max_depth);
        stats.playouts_total_depth += depth * ran;

        if (__builtin_expect(scheduler->cancelled(), 0)) {
            scheduler->yield();   // teardown: the main loop stops there (NetworkScheduler::cancel)
        } else if (conf->spin_yield_playouts > 0) {
            if (stats.num_evaluations != evals_seen) {   // (never after a spin run)
                evals_seen = stats.num_evaluations;
                quiet_playouts = 0;
            } else if ((quiet_playouts += ran) >= conf->spin_yield_playouts) {
                quiet_playouts = 0;
                scheduler->yield();
            }
        }
    }
}

// evaluator.cpp:888-943
PuctNode* PuctEvaluator::fastApplyMove(const PuctNodeChild* next) {
    GZ_ASSERT(root != nullptr && initial_root != nullptr);
    PuctNode* new_root = nullptr;
    for (int ii = 0; ii < root->num_children; ii++) {
        PuctNodeChild* c = root->getNodeChild(0, ii);
        if (c == next) {
            GZ_ASSERT(new_root == nullptr);
            if (c->to_node == nullptr) expandChild(root, c);
            new_root = c->to_node;
        } else if (c->to_node != nullptr) {
            PuctNode* next_node = c->to_node;
            c->to_node = nullptr;
            GZ_ASSERT(next_node->ref_count > 0);
            next_node->ref_count--;
            if (next_node->ref_count == 0) {
                releaseNodes(next_node);
                garbage.push_back(next_node);
            } else {
                detachEdge(c, next_node);
            }
        }
    }
    for (PuctNode* n : garbage) removeNode(n);
    garbage.clear();

    GZ_ASSERT(new_root != nullptr);
    root = new_root;
    root->in_parent = nullptr;   // a root's mirror is never read
    game_depth++;
    return root;
}

// evaluator.cpp:945-969
void PuctEvaluator::applyMove(const JointMove* move) {
    for (int ii = 0; ii < root->num_children; ii++) {
        PuctNodeChild* c = root->getNodeChild(0, ii);
        if (root->moveOf(c).equals(*move, sm->roleCount())) {
            fastApplyMove(c);
            break;
        }
    }
    GZ_ASSERT(root != nullptr);
}

// evaluator.cpp:971-1004
void PuctEvaluator::reset(int depth) {
    if (initial_root != nullptr) {
        releaseNodes(initial_root);
        garbage.push_back(initial_root);
        for (PuctNode* n : garbage) removeNode(n);
        garbage.clear();
        initial_root = root = nullptr;
    }
    stats.reset();
    game_depth = depth;
    mirror_ok = true;
}

// evaluator.cpp:1006-1017
PuctNode* PuctEvaluator::establishRoot(const uint64_t* current_state) {
    GZ_ASSERT(root == nullptr && initial_root == nullptr);
    if (current_state == nullptr) current_state = sm->initialState();
    initial_root = root = createNode(nullptr, current_state);
    GZ_ASSERT(!root->isTerminal());
    return root;
}

// evaluator.cpp:1019-1030
void PuctEvaluator::resetRootNode() {
    GZ_ASSERT(root != nullptr);
    for (int ii = 0; ii < root->num_children; ii++) {
        PuctNodeChild* c = root->getNodeChild(0, ii);
        c->policy_prob = c->policy_prob_orig;
        c->traversals = std::min(1U, c->traversals);
    }
    root->dirichlet_noise_set = false;
}

// evaluator.cpp:1032-1098
const PuctNodeChild* PuctEvaluator::onNextMove(int max_evaluations, double end_time) {
    GZ_ASSERT(root != nullptr && initial_root != nullptr);
    stats.reset();
    do_playouts = true;
    spin = SpinEpoch();   // the root changed (a freed root's address may be reused)

    if (conf->think_time > 10 && !root->dirichlet_noise_set && !root->is_finalised && root->visits > 10000) {
        if (number_of_nodes < 3000000) resetRootNode();
    }

    int worker_count = 0;
    auto f = [this, &worker_count]() {
        this->playoutWorker(worker_count);
        worker_count--;
    };
    if (conf->batch_size > 1 && root != nullptr && !root->is_finalised) {
        if (max_evaluations < 0 || max_evaluations > 100) {
            for (int ii = 0; ii < conf->batch_size - 1; ii++) {
                worker_count++;
                scheduler->addRunnable(f);
            }
        }
    }

    if (max_evaluations != 0) playoutMain(max_evaluations, end_time);

    do_playouts = false;
    while (worker_count > 0) scheduler->yield();

    return choose(root);
}

// evaluator.cpp:1100-1159
const PuctNodeChild* PuctEvaluator::chooseTopVisits(const PuctNode* node) const {
    GZ_ASSERT(node != nullptr);
    const PuctNodeChild* fast = nullptr;
    if (chooseTopVisitsFast(node, &fast)) {
        if (!verify_fastpath()) return fast;
        const PuctNodeChild* exact = chooseTopVisitsExact(node);
        if (exact != fast) {
            std::fprintf(stderr, "gz fast-path chooseTopVisits mismatch\n");
            std::abort();
        }
        return fast;
    }
    return chooseTopVisitsExact(node);
}

const PuctNodeChild* PuctEvaluator::chooseTopVisitsExact(const PuctNode* node) const {
    Children children = PuctNode::sortedChildrenTraversals(node);
    GZ_ASSERT(!children.empty());
    const int role_index = node->lead_role_index;
    int indx0 = -1, indx1 = -1;
    int count = 0;
    for (const PuctNodeChild* c : children) {
        if (c->to_node != nullptr && c->to_node->is_finalised) {
            if (c->to_node->getCurrentScore(role_index) > 0.99) return c;
            if (c->to_node->getCurrentScore(role_index) < 0.01) {
                count++;
                continue;
            }
        }
        if (indx0 == -1) indx0 = count;
        else if (indx1 == -1) indx1 = count;
        count++;
    }
    if (conf->top_visits_best_guess_converge_ratio > 0 && indx0 != -1 && indx1 != -1) {
        const PuctNodeChild* c0 = children[indx0];
        const PuctNodeChild* c1 = children[indx1];
        if (c0->to_node != nullptr && c1->to_node != nullptr) {
            if (c1->traversals > c0->traversals * conf->top_visits_best_guess_converge_ratio &&
                c1->to_node->getCurrentScore(role_index) > c0->to_node->getCurrentScore(role_index))
                return c1;
            return c0;
        }
    }
    return children[0];
}

// evaluator.cpp:1161-1192.  next_prob = pow(next_prob, temperature): the reference writes
// ::pow(float, float); this build evaluates it as the C library's double pow() and stores a float.
Children PuctEvaluator::getProbabilities(PuctNode* node, float temperature, bool use_policy) {
    GZ_ASSERT(node->num_children > 0);
    const float node_visits = node->visits + 0.001 * node->num_children;
    float total_probability = 0.0f;
    PuctChildCold* cold = node->cold();
    for (int ii = 0; ii < node->num_children; ii++) {
        PuctNodeChild* child = node->getNodeChild(0, ii);
        float& next_prob = cold[ii].next_prob;
        const float child_visits = child->to_node ? child->traversals + 0.001f : 0.001f;
        if (use_policy) next_prob = child->policy_prob + 0.001f;
        else next_prob = child_visits / node_visits;
        next_prob = (float)::pow((double)next_prob, (double)temperature);
        total_probability += next_prob;
    }
    for (int ii = 0; ii < node->num_children; ii++) cold[ii].next_prob /= total_probability;
    return PuctNode::sortedChildren(node, true);
}

// evaluator.cpp:1195-1224
float PuctEvaluator::priorScore(PuctNode* node, int depth) const {
    float prior_score = node->getFinalScore(node->lead_role_index);
    if (node->visits > 8) {
        const PuctNodeChild* best = chooseTopVisits(node);
        if (best->to_node != nullptr) prior_score = best->to_node->getCurrentScore(node->lead_role_index);
    }
    float fpu_reduction = depth == 0 ? conf->fpu_prior_discount_root : conf->fpu_prior_discount;
    if (fpu_reduction > 0) {
        float total_policy_visited = 0.0;
        for (int ii = 0; ii < node->num_children; ii++) {
            const PuctNodeChild* c = node->getNodeChild(0, ii);
            if (c->to_node != nullptr && c->to_node->visits > 0) total_policy_visited += c->policy_prob;
        }
        fpu_reduction *= std::sqrt(total_policy_visited);
        prior_score -= fpu_reduction;
    }
    return prior_score;
}

// evaluator.cpp:1227-1297
void PuctEvaluator::setDirichletNoise(PuctNode* node) {
    if (node->dirichlet_noise_set || node->num_children < 2 || conf->dirichlet_noise_pct < 0) return;
    if (node->getCurrentScore(node->lead_role_index) > 0.95) return;

    const float dirichlet_noise_alpha = 10.83f / node->num_children;
    std::gamma_distribution<float> gamma(dirichlet_noise_alpha, 1.0f);
    std::vector<float> dirichlet_noise(node->num_children, 0.0f);
    float total_noise = 0.0f;
    for (int ii = 0; ii < node->num_children; ii++) {
        const float noise = gamma(rng);
        dirichlet_noise[ii] = noise;
        total_noise += noise;
    }
    if (total_noise < std::numeric_limits<float>::min()) return;
    for (int ii = 0; ii < node->num_children; ii++) dirichlet_noise[ii] /= total_noise;

    const bool policy_squash = (conf->noise_policy_squash_pct > 0 && rng.get() < conf->noise_policy_squash_pct);
    float total_policy = 0;
    for (int ii = 0; ii < node->num_children; ii++) {
        PuctNodeChild* c = node->getNodeChild(0, ii);
        if (policy_squash) c->policy_prob = std::min(conf->noise_policy_squash_prob, c->policy_prob);
        const float pct = conf->dirichlet_noise_pct;
        c->policy_prob = (1.0f - pct) * c->policy_prob + pct * dirichlet_noise[ii];
        total_policy += c->policy_prob;
    }
    for (int ii = 0; ii < node->num_children; ii++) node->getNodeChild(0, ii)->policy_prob /= total_policy;
    node->dirichlet_noise_set = true;
}

// evaluator.cpp:1300-1307
void PuctEvaluator::setPuctConstant(PuctNode* node, int depth) const {
    const float puct_constant = depth == 0 ? conf->puct_constant_root : conf->puct_constant;
    node->puct_constant = puct_log(node->visits);
    node->puct_constant += puct_constant;
}

// evaluator.cpp:1309-1322
float PuctEvaluator::getTemperature(int depth) const {
    if (depth >= conf->depth_temperature_stop) return -1;
    float multiplier = 1.0f + ((depth - conf->depth_temperature_start) * conf->depth_temperature_increment);
    multiplier = std::max(1.0f, multiplier);
    return std::min(conf->temperature * multiplier, conf->depth_temperature_max);
}

// evaluator.cpp:1324-1340
const PuctNodeChild* PuctEvaluator::choose(const PuctNode* node) {
    if (conf->choose == ChooseFn::choose_temperature) return chooseTemperature(node);
    return chooseTopVisits(node);
}

// evaluator.cpp:1342-1362
bool PuctEvaluator::converged(int count) const {
    bool fast = false;
    if (convergedFast(count, &fast)) {
        if (verify_fastpath() && convergedExact(count) != fast) {
            std::fprintf(stderr, "gz fast-path converged mismatch\n");
            std::abort();
        }
        return fast;
    }
    return convergedExact(count);
}

bool PuctEvaluator::convergedExact(int count) const {
    Children children = PuctNode::sortedChildren(root);
    if (children.size() >= 2) {
        PuctNode* n0 = children[0]->to_node;
        PuctNode* n1 = children[1]->to_node;
        if (n0 != nullptr && n1 != nullptr) {
            const int role_index = root->lead_role_index;
            if (n0->getCurrentScore(role_index) > n1->getCurrentScore(role_index) && n0->visits > n1->visits + count)
                return true;
        }
        return false;
    }
    return true;
}

// evaluator.cpp:1473-1510
const PuctNodeChild* PuctEvaluator::chooseTemperature(const PuctNode* node) {
    if (node == nullptr) node = root;
    const float temperature = getTemperature(node->game_depth);
    if (temperature < 0) return chooseTopVisits(node);
    Children dist;
    if (conf->dirichlet_noise_pct < 0 && node->visits < 3) dist = getProbabilities(root, temperature, true);
    else dist = getProbabilities(root, temperature, false);
    const float expected_probability = rng.get() * conf->random_scale;
    float seen_probability = 0;
    for (const PuctNodeChild* c : dist) {
        seen_probability += root->coldOf(c).next_prob;
        if (seen_probability > expected_probability) return c;
    }
    return dist.back();
}

// node.cpp:400-441 (PuctNode::debug), sorted by traversals then lead-role score
void PuctEvaluator::nodeDebug(int child_index, int max_variation_depth, PuctNodeDebug& info) const {
    const PuctNode* node = root;
    if (node == nullptr || child_index >= node->num_children) return;
    Children node_children;
    for (int ii = 0; ii < node->num_children; ii++) node_children.push_back(node->getNodeChild(0, ii));
    const int ri = node->lead_role_index;
    std::sort(node_children.begin(), node_children.end(), [ri](const PuctNodeChild* a, const PuctNodeChild* b) {
        if (a->traversals != b->traversals) return a->traversals > b->traversals;
        const float a_prob = a->to_node != nullptr ? a->to_node->getCurrentScore(ri) : -1.0f;
        const float b_prob = b->to_node != nullptr ? b->to_node->getCurrentScore(ri) : -1.0f;
        return a_prob > b_prob;
    });
    const PuctNodeChild* child = node_children[child_index];
    if (child->to_node == nullptr) return;
    info.lead_role_index = node->lead_role_index;
    info.score = child->to_node->getCurrentScore(node->lead_role_index);
    info.move_index = node->moveOf(child).get(node->lead_role_index);
    const PuctNode* cur = child->to_node;
    for (int ii = 0; ii < max_variation_depth; ii++) {
        if (cur == nullptr || cur->num_children == 0 || cur->visits < 100) return;
        Children cc = PuctNode::sortedChildrenTraversals(cur, false);
        const PuctNodeChild* top = cc[0];
        info.variation.emplace_back(cur->lead_role_index, cur->moveOf(top).get(cur->lead_role_index));
        cur = top->to_node;
    }
}

}  // namespace gz
