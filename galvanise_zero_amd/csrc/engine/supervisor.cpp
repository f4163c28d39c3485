#include "supervisor.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace gz {

#define GZ_ASSERT(cond)                                                                     \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "gz assertion failed: %s (%s:%d)\n", #cond, __FILE__, __LINE__); \
            std::abort();                                                                   \
        }                                                                                   \
    } while (0)

// ---- Supervisor --------------------------------------------------------------------------------

Supervisor::Supervisor(const StateMachine* sm_, const GdlBasesTransformer* transformer, int batch_size,
                       std::string identifier, uint64_t seed, bool per_pool_unique_states)
    : sm(sm_->dupe()), transformer(transformer), batch_size(batch_size), identifier(std::move(identifier)),
      seed(seed), per_pool_unique_states(per_pool_unique_states),
      unique_states(transformer->createHashMask(sm_->numBases()), 1000) {}

Supervisor::~Supervisor() {
    for (SelfPlayWorker* w : self_play_workers) delete w;
    if (inline_sp_manager) delete inline_sp_manager;
    for (Sample* s : samples) delete s;
    for (UniqueStates* u : pool_unique_states) delete u;
    for (SelfPlayConfig* c : configs) delete c;
    delete sm;
}

UniqueStates* Supervisor::uniqueFor() {
    if (!per_pool_unique_states) return &unique_states;
    UniqueStates* u = new UniqueStates(transformer->createHashMask(sm->numBases()), 1000);
    pool_unique_states.push_back(u);
    return u;
}

// supervisor.cpp:43-66: every 1024 polls, report and move the pool's samples to the supervisor
void Supervisor::slowPoll(SelfPlayManager* manager) {
    slow_poll_counter++;
    if (slow_poll_counter < sample_interval) return;
    slow_poll_counter = 0;
    std::vector<Sample*>& other = manager->getSamples();
    if (other.empty()) return;
    std::lock_guard<std::mutex> lk(samples_m);
    samples.insert(samples.end(), other.begin(), other.end());
    other.clear();
}

// supervisor.cpp:68-77
void Supervisor::createInline(const SelfPlayConfig* config_in) {
    SelfPlayConfig* config = new SelfPlayConfig(*config_in);
    configs.push_back(config);
    inline_sp_manager = new SelfPlayManager(sm, transformer, batch_size, uniqueFor(), identifier + "_inline", seed,
                                            next_game_index);
    next_game_index += batch_size;
    all_managers.push_back(inline_sp_manager);
    inline_sp_manager->startSelfPlayers(config);
}

// supervisor.cpp:79-99
void Supervisor::createWorkers(const SelfPlayConfig* config_in) {
    SelfPlayConfig* config = new SelfPlayConfig(*config_in);
    configs.push_back(config);
    const int count = (int)self_play_workers.size() * 2;
    SelfPlayManager* m0 = new SelfPlayManager(sm, transformer, batch_size, uniqueFor(),
                                              identifier + "_sp" + std::to_string(count), seed, next_game_index);
    next_game_index += batch_size;
    SelfPlayManager* m1 = new SelfPlayManager(sm, transformer, batch_size, uniqueFor(),
                                              identifier + "_sp" + std::to_string(count + 1), seed, next_game_index);
    next_game_index += batch_size;
    all_managers.push_back(m0);
    all_managers.push_back(m1);
    self_play_workers.push_back(new SelfPlayWorker(this, m0, m1, config));
}

// supervisor.cpp:101-168
void Supervisor::cancel() {
    cancelled.store(true);
    for (SelfPlayManager* m : all_managers) m->cancel();
    {
        std::lock_guard<std::mutex> lk(ready_m);
        ready_flag++;
    }
    ready_cv.notify_all();
}

const ReadyEvent* Supervisor::poll(int predict_count, const std::vector<float*>& data) {
    GZ_ASSERT(0 <= predict_count && predict_count <= batch_size);
    if (cancelled.load()) return &cancelled_event;

    auto populateEvent = [&](SelfPlayManager* manager) {
        PredictDoneEvent* event = manager->getPredictDoneEvent();
        event->pred_count = predict_count;
        if (predict_count > 0) {
            int index = 0;
            for (int ii = 0; ii < transformer->getNumberPolicies(); ii++)
                std::memcpy(event->policies[ii], data[index++],
                            sizeof(float) * predict_count * transformer->getPolicySize(ii));
            std::memcpy(event->final_scores, data[index++], sizeof(float) * predict_count * transformer->getNumberRewards());
        }
    };

    if (inline_sp_manager != nullptr) {
        populateEvent(inline_sp_manager);
        inline_sp_manager->poll();
        slowPoll(inline_sp_manager);
        return inline_sp_manager->getReadyEvent();
    }

    GZ_ASSERT(!self_play_workers.empty());
    if (predict_count) {
        GZ_ASSERT(in_progress_worker != nullptr && in_progress_manager != nullptr);
        populateEvent(in_progress_manager);
        slowPoll(in_progress_manager);
        in_progress_worker->push(in_progress_manager);
        in_progress_worker = nullptr;
        in_progress_manager = nullptr;
    }
    GZ_ASSERT(in_progress_worker == nullptr && in_progress_manager == nullptr);

    // wait for any worker to hand back a pool (the reference busy-spins, supervisor.cpp:146-165)
    while (true) {
        long seen;
        {
            std::lock_guard<std::mutex> lk(ready_m);
            seen = ready_flag;
        }
        for (SelfPlayWorker* worker : self_play_workers) {
            in_progress_manager = worker->pull();
            if (in_progress_manager != nullptr) {
                in_progress_worker = worker;
                break;
            }
        }
        if (in_progress_worker != nullptr) break;
        if (cancelled.load()) return &cancelled_event;
        std::unique_lock<std::mutex> lk(ready_m);
        ready_cv.wait(lk, [&] { return ready_flag != seen; });
    }
    return in_progress_manager->getReadyEvent();
}

std::vector<Sample*> Supervisor::getSamples() {
    std::lock_guard<std::mutex> lk(samples_m);
    std::vector<Sample*> result = std::move(samples);
    samples.clear();
    return result;
}

void Supervisor::clearUniqueStates() {
    unique_states.clear();
    for (UniqueStates* u : pool_unique_states) u->clear();
}

PoolStats Supervisor::stats() {
    PoolStats s;
    for (SelfPlayManager* m : all_managers) {
        const PoolStats& p = m->getStats();
        s.games_started += p.games_started;
        s.games_completed += p.games_completed;
        s.games_with_samples += p.games_with_samples;
        s.samples += p.samples;
        s.no_samples += p.no_samples;
        s.dupes += p.dupes;
        s.resigns += p.resigns;
        s.false_positive_resigns0 += p.false_positive_resigns0;
        s.false_positive_resigns1 += p.false_positive_resigns1;
        s.early_run_to_ends += p.early_run_to_ends;
        s.aborts_game_length += p.aborts_game_length;
        s.evaluations += p.evaluations;
        s.polls += p.polls;
        s.completed_game_evals += p.completed_game_evals;
        s.tree_playouts += m->treePlayouts();
        s.transpositions += m->transpositions();
    }
    return s;
}

// ---- SelfPlayWorker (supervisor.cpp:183-245) ------------------------------------------------

SelfPlayWorker::SelfPlayWorker(Supervisor* sup, SelfPlayManager* man0, SelfPlayManager* man1,
                               const SelfPlayConfig* config)
    : sup(sup), man0(man0), man1(man1), config(config) {
    thread = std::thread([this]() { this->run(); });
}

SelfPlayWorker::~SelfPlayWorker() {
    stop = true;
    // a pool can spin for minutes without an evaluation (the reference's playoutMain): cancel both
    // so that a poll in progress returns at its games' next yield instead of at their next batch
    man0->cancel();
    man1->cancel();
    inbound.wake();
    if (thread.joinable()) thread.join();
    delete man0;
    delete man1;
}

void SelfPlayWorker::run() {
    // prime both pools (each runs until its first batch is ready)
    for (SelfPlayManager* m : {man0, man1}) {
        m->startSelfPlayers(config);
        m->getPredictDoneEvent()->pred_count = 0;
        m->poll();
        outbound.push(m);
        sup->notifyReady();
    }
    while (!stop) {
        SelfPlayManager* m = nullptr;
        if (!inbound.popWait(m, stop)) continue;
        m->poll();
        outbound.push(m);
        sup->notifyReady();
    }
}

// ---- Player (player.cpp) ----------------------------------------------------------------------

Player::Player(const StateMachine* sm_, const GdlBasesTransformer* transformer, const PuctConfig& conf, uint64_t seed)
    : sm(sm_->dupe()), transformer(transformer), config(conf) {
    GZ_ASSERT(config.batch_size >= 1);
    scheduler = new NetworkScheduler(transformer, config.batch_size);
    evaluator = new PuctEvaluator(sm, scheduler, transformer);
    evaluator->updateConf(&config);
    evaluator->seed(Rng::mix(seed, 0, 0));
}

Player::~Player() {
    delete evaluator;
    delete scheduler;
    delete sm;
}

void Player::updateConfig(float think_time, int converged_visits, bool verbose) {
    config.think_time = think_time;
    config.converged_visits = converged_visits;
    config.verbose = verbose;
    evaluator->updateConf(&config);
}

void Player::puctPlayerReset(int game_depth) {
    evaluator->reset(game_depth);
    first_play = true;
}

void Player::puctApplyMove(const JointMove& move) {
    scheduler->createMainLoop();
    pending_move = move;
    if (first_play) {
        first_play = false;
        scheduler->addRunnable([this]() {
            evaluator->establishRoot(nullptr);
            evaluator->applyMove(&pending_move);
        });
    } else {
        scheduler->addRunnable([this]() { evaluator->applyMove(&pending_move); });
    }
}

void Player::puctPlayerMove(const uint64_t* state, int evaluations, double end_time) {
    on_next_move_choice = nullptr;
    scheduler->createMainLoop();
    if (first_play) {
        first_play = false;
        pending_state.assign(state, state + sm->numWords());
        scheduler->addRunnable([this, evaluations, end_time]() {
            evaluator->establishRoot(pending_state.data());
            on_next_move_choice = evaluator->onNextMove(evaluations, end_time);
        });
    } else {
        scheduler->addRunnable([this, evaluations, end_time]() {
            on_next_move_choice = evaluator->onNextMove(evaluations, end_time);
        });
    }
}

std::tuple<int, float, int> Player::puctPlayerGetMove(int lead_role_index) {
    if (on_next_move_choice == nullptr) return std::make_tuple(-1, -1.0f, -1);
    float probability = -1;
    const PuctNode* node = on_next_move_choice->to_node;
    if (node != nullptr) probability = node->getCurrentScore(lead_role_index);
    // (the choice is a child entry of the current root: onNextMove returned it, no move applied since)
    const JointMove& move = evaluator->getRootNode()->moveOf(on_next_move_choice);
    return std::make_tuple(move.get(lead_role_index), probability, evaluator->nodeCount());
}

void Player::balanceNode(int max_count) {
    scheduler->createMainLoop();
    const PuctNode* root = evaluator->getRootNode();
    if (root == nullptr) return;
    max_count = std::min((int)root->num_children, max_count);
    scheduler->addRunnable([this, max_count]() { evaluator->balanceFirstMoves(max_count); });
}

std::vector<PuctNodeDebug> Player::treeDebugInfo(int max_count) {
    std::vector<PuctNodeDebug> res;
    const PuctNode* root = evaluator->getRootNode();
    if (root == nullptr) return res;
    max_count = std::min((int)root->num_children, max_count);
    for (int ii = 0; ii < max_count; ii++) {
        PuctNodeDebug info;
        evaluator->nodeDebug(ii, 10, info);
        res.push_back(info);
    }
    return res;
}

// player.cpp:155-173: stores the caller's array pointers (caller keeps them alive until next poll)
const ReadyEvent* Player::poll(int predict_count, const std::vector<float*>& data) {
    predict_done_event.pred_count = predict_count;
    int index = 0;
    predict_done_event.policies.resize(transformer->getNumberPolicies());
    for (int ii = 0; ii < transformer->getNumberPolicies(); ii++) predict_done_event.policies[ii] = data[index++];
    predict_done_event.final_scores = data[index++];
    if (!scheduler->hasMainLoop()) {
        ready_event.buf_count = 0;
        return &ready_event;
    }
    scheduler->poll(&predict_done_event, &ready_event);
    return &ready_event;
}

}  // namespace gz
