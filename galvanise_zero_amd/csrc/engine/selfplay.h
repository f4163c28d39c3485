// Self-play game driver, sample records, duplicate-state filter and game pool.  Restates
//   SelfPlay          reference src/cpp/selfplay.h:43-91, selfplay.cpp:29-343
//   Sample            src/cpp/sample.h:12-29
//   UniqueStates      src/cpp/uniquestates.h:14-79
//   SelfPlayManager   src/cpp/selfplaymanager.h:19-113, selfplaymanager.cpp:22-200
#pragma once

#include "config.h"
#include "evaluator.h"
#include "scheduler.h"
#include "sm.h"
#include "transformer.h"

#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace gz {

struct Sample {
    typedef std::vector<std::pair<int, float>> Policy;
    std::vector<uint64_t> state;
    std::vector<std::vector<uint64_t>> prev_states;
    std::vector<Policy> policies;
    std::vector<float> final_score;
    int depth = 0;
    int game_length = 0;
    std::string match_identifier;
    bool has_resigned = false;
    bool resign_false_positive = false;
    int starting_sample_depth = 0;
    std::vector<float> resultant_puct_score;
    int resultant_puct_visits = 0;
    int lead_role_index = 0;
};

// uniquestates.h: thread-safe (mutex) count of states seen, keyed by the transformer's base mask.
class UniqueStates {
public:
    UniqueStates(const std::vector<uint64_t>& mask, int max_num_dupes = 1) : mask(mask), max_num_dupes(max_num_dupes) {}
    void add(const uint64_t* bs);
    bool isUnique(const uint64_t* bs, int depth);
    void clear();

private:
    struct Key {
        std::vector<uint64_t> w;
        bool operator==(const Key& o) const { return w == o.w; }
    };
    struct Hash {
        size_t operator()(const Key& k) const;
    };
    Key key(const uint64_t* bs) const;

    std::vector<uint64_t> mask;
    const int max_num_dupes;
    std::mutex mut;
    std::unordered_map<Key, int, Hash> lookup;
};

class SelfPlayManager;

class SelfPlay {
public:
    SelfPlay(SelfPlayManager* manager, const SelfPlayConfig* conf, PuctEvaluator* pe,
             const uint64_t* initial_state, int role_count, std::string identifier, uint64_t seed);
    void playOnce();
    void playGamesForever();
    int matchCount() const { return match_count; }   // games started (the current one included)

private:
    bool resign(const PuctNode* node);
    PuctNode* collectSamples(PuctNode* node);
    int runToEnd(PuctNode* node, std::vector<float>& final_scores);
    void addSamples(const std::vector<float>& final_scores, int starting_sample_depth, int game_depth);
    bool checkFalsePositive(const std::vector<float>& scores, float resign_probability, float final_score, int role_index);

    SelfPlayManager* manager;
    const SelfPlayConfig* conf;
    PuctEvaluator* pe;
    const uint64_t* initial_state;
    const int role_count;
    const std::string identifier;
    int match_count = 0;
    std::vector<Sample*> game_samples;
    bool has_resigned = false;
    bool can_resign0 = false;
    bool can_resign1 = false;
    std::vector<float> resign0_false_positive_check_scores;
    std::vector<float> resign1_false_positive_check_scores;
    Rng rng;

public:
    // the game in progress (diagnostics, read racily by stats snapshots): its coroutine, and the
    // coroutine's TSC cycles / the evaluator's evaluations when it started
    const Coro* coro = nullptr;
    uint64_t game_c0 = 0;
    long game_e0 = 0;
};

// Per-game cost by the game's ordinal within its slot (1st, 2nd, ... game a SelfPlay plays; the
// last bucket holds every later one): is a slot's k-th game more expensive than its first?
struct OrdinalStats {
    static constexpr int kOrdinals = 8, kHist = 32;
    long games[kOrdinals] = {};
    long evals[kOrdinals] = {};
    long tree_playouts[kOrdinals] = {};
    long moves[kOrdinals] = {};
    long spin_epochs[kOrdinals] = {};
    uint64_t cycles[kOrdinals] = {};
    long cost_hist[kHist] = {};    // completed games by engine milliseconds, [2^(k-1), 2^k) ms
};

struct PoolStats {
    long games_started = 0;        // playOnce() calls
    long games_completed = 0;      // playOnce() returns (incl. no-sample restarts and aborts)
    long games_with_samples = 0;   // games that emitted samples (= distinct match_identifier)
    long samples = 0;
    long no_samples = 0;
    long dupes = 0;
    long resigns = 0;
    long false_positive_resigns0 = 0;
    long false_positive_resigns1 = 0;
    long early_run_to_ends = 0;
    long aborts_game_length = 0;
    long evaluations = 0;          // NN rows requested
    long polls = 0;
    long completed_game_evals = 0; // NN evaluations consumed by the games counted in games_completed
    long tree_playouts = 0;        // tree playouts of every game of the pool (filled by treePlayouts())
    long transpositions = 0;       // transposition edges attached (filled by transpositions())
    OrdinalStats ord;
};

class SelfPlayManager {
public:
    // game_index_base / seed: game i of this pool uses RNG streams derived from
    // (seed, game_index_base + i), independent of pool / thread / GPU placement.
    SelfPlayManager(const StateMachine* sm, const GdlBasesTransformer* transformer, int batch_size,
                    UniqueStates* unique_states, std::string identifier, uint64_t seed, long game_index_base,
                    float* channel_buf = nullptr, float* const* policy_bufs = nullptr, float* value_buf = nullptr);
    ~SelfPlayManager();

    Sample* createSample(const PuctEvaluator* pe, const PuctNode* node);
    void addSample(Sample* sample);
    UniqueStates* getUniqueStates() const { return unique_states; }

    void incrDupes() { stats.dupes++; }
    void incrNoSamples() { stats.no_samples++; }
    void incrResign0FalsePositives() { stats.false_positive_resigns0++; }
    void incrResign1FalsePositives() { stats.false_positive_resigns1++; }
    void incrEarlyRunToEnds() { stats.early_run_to_ends++; }
    void incrResigns() { stats.resigns++; }
    void incrAbortsGameLength() { stats.aborts_game_length++; }
    PoolStats& getStats() { return stats; }
    long treePlayouts() const {
        long n = 0;
        for (const PuctEvaluator* pe : evaluators) n += pe->totalTreePlayouts();
        return n;
    }
    long transpositions() const {
        long n = 0;
        for (const PuctEvaluator* pe : evaluators) n += pe->totalTranspositions();
        return n;
    }

    void startSelfPlayers(const SelfPlayConfig* config);
    void poll();
    // teardown from any thread: the pool's poll returns promptly with no rows (NetworkScheduler::cancel)
    void cancel() { scheduler->cancel(); }

    // games in progress by ordinal (OrdinalStats::kOrdinals buckets): count, engine seconds and
    // evaluations they have used so far
    void inflight(long* games, double* engine_s, long* evals) const;

    std::vector<Sample*>& getSamples() { return samples; }
    ReadyEvent* getReadyEvent() { return &ready_event; }
    PredictDoneEvent* getPredictDoneEvent() { return &predict_done_event; }
    int batchSize() const { return batch_size; }
    const GdlBasesTransformer* getTransformer() const { return transformer; }

private:
    StateMachine* sm;
    const GdlBasesTransformer* transformer;
    int batch_size;
    std::vector<SelfPlay*> self_plays;
    std::vector<PuctEvaluator*> evaluators;
    NetworkScheduler* scheduler;
    std::vector<Sample*> samples;
    UniqueStates* unique_states;
    std::string identifier;
    uint64_t seed;
    long game_index_base;
    ReadyEvent ready_event;
    PredictDoneEvent predict_done_event;
    bool owns_pred_bufs = true;
    PoolStats stats;
};

}  // namespace gz
