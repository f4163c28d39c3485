// Supervisor (reference src/cpp/supervisor.h:65-109, supervisor.cpp:19-168): owns the game pools
// (inline in the polling thread, or worker threads each ping-ponging two pools, supervisor.cpp:
// 79-99, 196-245) behind the poll(predict_count, arrays) protocol; and Player (player.h:19-57,
// player.cpp): one evaluator + one scheduler for match play behind the same protocol.
#pragma once

#include "evaluator.h"
#include "selfplay.h"

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <tuple>

namespace gz {

template <typename T>
class LockedQueue {
public:
    void push(T v) {
        {
            std::lock_guard<std::mutex> lk(m);
            q.push_back(v);
        }
        cv.notify_one();
    }
    bool tryPop(T& out) {
        std::lock_guard<std::mutex> lk(m);
        if (q.empty()) return false;
        out = q.front();
        q.pop_front();
        return true;
    }
    bool popWait(T& out, const std::atomic<bool>& stop) {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return !q.empty() || stop.load(); });
        if (q.empty()) return false;
        out = q.front();
        q.pop_front();
        return true;
    }
    void wake() { cv.notify_all(); }

private:
    std::mutex m;
    std::condition_variable cv;
    std::deque<T> q;
};

class Supervisor;

class SelfPlayWorker {
public:
    SelfPlayWorker(Supervisor* sup, SelfPlayManager* man0, SelfPlayManager* man1, const SelfPlayConfig* config);
    ~SelfPlayWorker();
    SelfPlayManager* pull() {
        SelfPlayManager* m = nullptr;
        return outbound.tryPop(m) ? m : nullptr;
    }
    void push(SelfPlayManager* m) { inbound.push(m); }

private:
    void run();
    Supervisor* sup;
    SelfPlayManager* man0;
    SelfPlayManager* man1;
    const SelfPlayConfig* config;
    LockedQueue<SelfPlayManager*> inbound;
    LockedQueue<SelfPlayManager*> outbound;
    std::atomic<bool> stop{false};
    std::thread thread;
    friend class Supervisor;
};

class Supervisor {
public:
    Supervisor(const StateMachine* sm, const GdlBasesTransformer* transformer, int batch_size, std::string identifier,
               uint64_t seed = 0, bool per_pool_unique_states = false);
    ~Supervisor();

    void createInline(const SelfPlayConfig* config);
    void createWorkers(const SelfPlayConfig* config);

    std::vector<Sample*> getSamples();
    const ReadyEvent* poll(int predict_count, const std::vector<float*>& data);

    void addUniqueState(const uint64_t* bs) { unique_states.add(bs); }
    // polls between sample collections (reference: 1024, supervisor.cpp:45)
    void setSampleInterval(int n) { sample_interval = n < 1 ? 1 : n; }
    void clearUniqueStates();
    PoolStats stats();
    // Bounded teardown (any thread, also while another thread is inside poll()): every pool is
    // cancelled (NetworkScheduler::cancel) and poll() returns an empty batch from then on.
    void cancel();

    // called by workers when a pool is ready
    void notifyReady() {
        {
            std::lock_guard<std::mutex> lk(ready_m);
            ready_flag++;
        }
        ready_cv.notify_one();
    }

private:
    void slowPoll(SelfPlayManager* manager);
    UniqueStates* uniqueFor();

    StateMachine* sm;
    const GdlBasesTransformer* transformer;
    const int batch_size;
    const std::string identifier;
    const uint64_t seed;
    const bool per_pool_unique_states;
    int slow_poll_counter = 0;
    int sample_interval = 1024;
    long next_game_index = 0;

    std::atomic<bool> cancelled{false};
    ReadyEvent cancelled_event;        // the empty batch poll() returns once cancelled
    SelfPlayManager* inline_sp_manager = nullptr;
    SelfPlayManager* in_progress_manager = nullptr;
    SelfPlayWorker* in_progress_worker = nullptr;
    std::vector<SelfPlayWorker*> self_play_workers;
    std::vector<SelfPlayManager*> all_managers;
    std::vector<SelfPlayConfig*> configs;

    std::mutex samples_m;
    std::vector<Sample*> samples;
    UniqueStates unique_states;
    std::vector<UniqueStates*> pool_unique_states;

    std::mutex ready_m;
    std::condition_variable ready_cv;
    long ready_flag = 0;
};

class Player {
public:
    Player(const StateMachine* sm, const GdlBasesTransformer* transformer, const PuctConfig& conf, uint64_t seed = 0);
    ~Player();

    void updateConfig(float think_time, int converged_visits, bool verbose);
    void puctPlayerReset(int game_depth);
    void puctApplyMove(const JointMove& move);
    void puctPlayerMove(const uint64_t* state, int evaluations, double end_time);
    std::tuple<int, float, int> puctPlayerGetMove(int lead_role_index);
    void balanceNode(int max_count);
    std::vector<PuctNodeDebug> treeDebugInfo(int max_count);
    const ReadyEvent* poll(int predict_count, const std::vector<float*>& data);
    PuctEvaluator* getEvaluator() { return evaluator; }

private:
    StateMachine* sm;
    const GdlBasesTransformer* transformer;
    PuctConfig config;
    PuctEvaluator* evaluator;
    NetworkScheduler* scheduler;
    bool first_play = false;
    const PuctNodeChild* on_next_move_choice = nullptr;
    JointMove pending_move{};
    std::vector<uint64_t> pending_state;
    ReadyEvent ready_event;
    PredictDoneEvent predict_done_event;
};

}  // namespace gz
