#include "selfplay.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace gz {

#define GZ_ASSERT(cond)                                                                     \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "gz assertion failed: %s (%s:%d)\n", #cond, __FILE__, __LINE__); \
            std::abort();                                                                   \
        }                                                                                   \
    } while (0)

// ---- UniqueStates (uniquestates.h:28-76) --------------------------------------------------------

size_t UniqueStates::Hash::operator()(const Key& k) const {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint64_t w : k.w) h ^= w + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    return (size_t)h;
}

UniqueStates::Key UniqueStates::key(const uint64_t* bs) const {
    Key k;
    k.w.resize(mask.size());
    for (size_t i = 0; i < mask.size(); ++i) k.w[i] = bs[i] & mask[i];
    return k;
}

void UniqueStates::add(const uint64_t* bs) {
    std::lock_guard<std::mutex> lk(mut);
    Key k = key(bs);
    auto it = lookup.find(k);
    if (it != lookup.end()) {
        if (it->second < max_num_dupes) it->second += 1;
        return;
    }
    lookup.emplace(std::move(k), 1);
}

bool UniqueStates::isUnique(const uint64_t* bs, int depth) {
    std::lock_guard<std::mutex> lk(mut);
    auto it = lookup.find(key(bs));
    if (it != lookup.end()) {
        const int allowed_dupes = std::max(2, (max_num_dupes - 5 * depth));
        if (it->second >= allowed_dupes) return false;
    }
    return true;
}

void UniqueStates::clear() {
    std::lock_guard<std::mutex> lk(mut);
    lookup.clear();
}

// ---- SelfPlay (selfplay.cpp) --------------------------------------------------------------------

SelfPlay::SelfPlay(SelfPlayManager* manager, const SelfPlayConfig* conf, PuctEvaluator* pe,
                   const uint64_t* initial_state, int role_count, std::string identifier, uint64_t seed)
    : manager(manager), conf(conf), pe(pe), initial_state(initial_state), role_count(role_count),
      identifier(std::move(identifier)), rng(seed) {}

// selfplay.cpp:43-74
bool SelfPlay::resign(const PuctNode* node) {
    GZ_ASSERT(!node->isTerminal());
    GZ_ASSERT(!has_resigned);
    const float score = node->getCurrentScore(node->lead_role_index);
    if (can_resign0 && score < conf->resign0_score_probability) {
        has_resigned = true;
        for (int ii = 0; ii < role_count; ii++) resign0_false_positive_check_scores.push_back(node->getCurrentScore(ii));
    } else if (can_resign1 && score < conf->resign1_score_probability) {
        has_resigned = true;
        for (int ii = 0; ii < role_count; ii++) resign1_false_positive_check_scores.push_back(node->getCurrentScore(ii));
    }
    return has_resigned;
}

// selfplay.cpp:76-169
PuctNode* SelfPlay::collectSamples(PuctNode* node) {
    pe->updateConf(&conf->puct_config);
    const bool do_oscillate_sampling = conf->oscillate_sampling_pct > 0;
    const int evals = conf->evals_per_move;
    UniqueStates& man = *manager->getUniqueStates();

    while (true) {
        if (conf->abort_max_length > 0 && node->game_depth > conf->abort_max_length) break;
        if (node->isTerminal()) break;

        const PuctNodeChild* choice = nullptr;
        bool do_skip = false;
        if (!man.isUnique(node->getBaseState(), node->game_depth)) {
            manager->incrDupes();
            do_skip = true;
        } else {
            if (do_oscillate_sampling && rng.get() > conf->oscillate_sampling_pct) do_skip = true;
        }

        if (!do_skip) {
            man.add(node->getBaseState());
            pe->resetRootNode();
            choice = pe->onNextMove(evals);
            pe->getProbabilities(node, conf->temperature_for_policy, false);
            Sample* s = manager->createSample(pe, node);
            game_samples.push_back(s);
        } else {
            const int skip_evals = std::max(16, (int)rng.getWithMax(evals / 3 + 1));
            pe->updateConf(&conf->run_to_end_puct_config);
            choice = pe->onNextMove(skip_evals);
            pe->updateConf(&conf->puct_config);
        }

        GZ_ASSERT(choice != nullptr);
        node = pe->fastApplyMove(choice);
        if (node->isTerminal()) break;
        if (!has_resigned) resign(node);
        if (has_resigned && game_samples.size() > 1) {
            manager->incrResigns();
            break;
        }
    }
    return node;
}

// selfplay.cpp:171-228
int SelfPlay::runToEnd(PuctNode* node, std::vector<float>& final_scores) {
    pe->updateConf(&conf->run_to_end_puct_config);
    const int evals = conf->run_to_end_evals;
    const bool run_to_end_can_resign = (has_resigned && rng.get() > conf->run_to_end_pct);

    auto done = [this](const PuctNode* n) {
        if (conf->abort_max_length > 0 && n->game_depth > conf->abort_max_length) return true;
        return n->is_finalised;
    };

    while (!done(node)) {
        const PuctNodeChild* choice = pe->onNextMove(evals);
        node = pe->fastApplyMove(choice);
        if (node->is_finalised) break;
        if (run_to_end_can_resign && node->game_depth > conf->run_to_end_minimum_game_depth) {
            const float lead_score = node->getCurrentScore(node->lead_role_index);
            if (lead_score < conf->run_to_end_early_score) {
                manager->incrEarlyRunToEnds();
                for (int ri = 0; ri < role_count; ri++) final_scores.push_back(ri == node->lead_role_index ? 0.0 : 1.0);
                return node->game_depth;
            }
        }
    }
    if (conf->abort_max_length > 0 && node->game_depth > conf->abort_max_length) return -1;
    for (int ri = 0; ri < role_count; ri++) final_scores.push_back(node->getCurrentScore(ri));
    return node->game_depth;
}

// selfplay.cpp:230-247
bool SelfPlay::checkFalsePositive(const std::vector<float>& scores, float resign_probability, float final_score,
                                  int role_index) {
    if (!scores.empty()) {
        const float score = scores[role_index];
        if ((score < resign_probability * 1.05) && final_score > 0.49) return true;
    }
    return false;
}

// selfplay.cpp:249-288
void SelfPlay::addSamples(const std::vector<float>& final_scores, int starting_sample_depth, int game_depth) {
    bool is_resign0_false_positive = false;
    bool is_resign1_false_positive = false;
    for (int ri = 0; ri < role_count; ri++) {
        const float final_score = final_scores[ri];
        if (has_resigned) {
            if (!is_resign0_false_positive &&
                checkFalsePositive(resign0_false_positive_check_scores, conf->resign0_score_probability, final_score, ri)) {
                is_resign0_false_positive = true;
                manager->incrResign0FalsePositives();
            }
            if (!is_resign1_false_positive &&
                checkFalsePositive(resign1_false_positive_check_scores, conf->resign1_score_probability, final_score, ri)) {
                is_resign1_false_positive = true;
                manager->incrResign1FalsePositives();
            }
        }
    }
    for (Sample* sample : game_samples) {
        sample->final_score = final_scores;
        sample->game_length = game_depth;
        sample->match_identifier = identifier + "_" + std::to_string(match_count);
        sample->has_resigned = has_resigned;
        sample->resign_false_positive = is_resign0_false_positive || is_resign1_false_positive;
        sample->starting_sample_depth = starting_sample_depth;
        manager->addSample(sample);
    }
    manager->getStats().games_with_samples++;
}

// selfplay.cpp:292-337
void SelfPlay::playOnce() {
    match_count++;
    manager->getStats().games_started++;
    game_samples.clear();
    has_resigned = false;
    const double r = rng.get();
    can_resign0 = r > conf->resign0_pct;
    can_resign1 = r > conf->resign1_pct;
    resign0_false_positive_check_scores.clear();
    resign1_false_positive_check_scores.clear();

    const long evals0 = pe->totalEvaluations();
    const long playouts0 = pe->totalTreePlayouts();
    const long epochs0 = pe->totalSpinEpochs();
    coro = coro_current();
    game_e0 = evals0;
    game_c0 = coro_cycles_now();
    int starting_sample_depth = 0;
    auto completed = [&]() {
        PoolStats& st = manager->getStats();
        st.games_completed++;
        st.completed_game_evals += pe->totalEvaluations() - evals0;
        OrdinalStats& o = st.ord;
        const int k = std::min(match_count, OrdinalStats::kOrdinals) - 1;
        const uint64_t cyc = coro_cycles_now() - game_c0;
        o.games[k]++;
        o.evals[k] += pe->totalEvaluations() - evals0;
        o.tree_playouts[k] += pe->totalTreePlayouts() - playouts0;
        o.moves[k] += pe->getRootNode()->game_depth - starting_sample_depth;
        o.spin_epochs[k] += pe->totalSpinEpochs() - epochs0;
        o.cycles[k] += cyc;
        const double ms = (double)cyc / tsc_hz() * 1e3;
        int b = 0;
        while (b < OrdinalStats::kHist - 1 && ms >= (double)(1L << b)) ++b;
        o.cost_hist[b]++;
    };

    pe->reset(0);
    PuctNode* node = pe->establishRoot(initial_state);
    GZ_ASSERT(!node->isTerminal());
    starting_sample_depth = node->game_depth;

    node = collectSamples(node);
    if (game_samples.empty()) {
        manager->incrNoSamples();
        completed();
        return;
    }

    std::vector<float> final_scores;
    const int game_depth = runToEnd(node, final_scores);
    completed();
    if (game_depth == -1) {
        for (Sample* s : game_samples) delete s;
        game_samples.clear();
        manager->incrAbortsGameLength();
        return;
    }
    addSamples(final_scores, starting_sample_depth, game_depth);
}

void SelfPlay::playGamesForever() {
    while (true) playOnce();
}

// ---- SelfPlayManager (selfplaymanager.cpp) ------------------------------------------------------

SelfPlayManager::SelfPlayManager(const StateMachine* sm_, const GdlBasesTransformer* transformer, int batch_size,
                                 UniqueStates* unique_states, std::string identifier, uint64_t seed,
                                 long game_index_base, float* channel_buf, float* const* policy_bufs,
                                 float* value_buf)
    : sm(sm_->dupe()), transformer(transformer), batch_size(batch_size), unique_states(unique_states),
      identifier(std::move(identifier)), seed(seed), game_index_base(game_index_base) {
    scheduler = new NetworkScheduler(transformer, batch_size, channel_buf);
    if (policy_bufs != nullptr) {
        owns_pred_bufs = false;
        for (int ii = 0; ii < transformer->getNumberPolicies(); ii++) predict_done_event.policies.push_back(policy_bufs[ii]);
        predict_done_event.final_scores = value_buf;
    } else {
        for (int ii = 0; ii < transformer->getNumberPolicies(); ii++)
            predict_done_event.policies.push_back(new float[(size_t)transformer->getPolicySize(ii) * batch_size]);
        predict_done_event.final_scores = new float[(size_t)transformer->getNumberRewards() * batch_size];
    }
    predict_done_event.pred_count = 0;
}

SelfPlayManager::~SelfPlayManager() {
    delete scheduler;   // destroys the (suspended) game coroutines first
    for (SelfPlay* sp : self_plays) delete sp;
    for (PuctEvaluator* pe : evaluators) delete pe;
    for (Sample* s : samples) delete s;
    if (owns_pred_bufs) {
        for (float* mem : predict_done_event.policies) delete[] mem;
        delete[] predict_done_event.final_scores;
    }
    delete sm;
}

// selfplaymanager.cpp:72-119
Sample* SelfPlayManager::createSample(const PuctEvaluator* pe, const PuctNode* node) {
    Sample* sample = new Sample;
    const int nw = sm->numWords();
    sample->state.assign(node->getBaseState(), node->getBaseState() + nw);
    const PuctNode* cur = node->parent;
    for (int ii = 0; ii < transformer->getNumberPrevStates(); ii++) {
        if (cur == nullptr) break;
        sample->prev_states.emplace_back(cur->getBaseState(), cur->getBaseState() + nw);
        cur = cur->parent;
    }
    const int role_count = sm->roleCount();
    sample->policies.resize(role_count);
    for (int ri = 0; ri < role_count; ri++) {
        Sample::Policy& policy = sample->policies[ri];
        for (int ii = 0; ii < node->num_children; ii++) {
            const PuctChildCold& cold = node->cold()[ii];
            if (ri == node->lead_role_index) {
                policy.emplace_back(cold.move.get(ri), cold.next_prob);
            } else {
                policy.emplace_back(cold.move.get(ri), 1.0f);
                break;
            }
        }
    }
    sample->resultant_puct_visits = node->visits;
    for (int ii = 0; ii < role_count; ii++) sample->resultant_puct_score.push_back(node->getCurrentScore(ii));
    sample->depth = node->game_depth;
    sample->lead_role_index = node->lead_role_index;
    (void)pe;
    return sample;
}

void SelfPlayManager::addSample(Sample* sample) {
    samples.push_back(sample);
    stats.samples++;
}

// selfplaymanager.cpp:127-150
void SelfPlayManager::startSelfPlayers(const SelfPlayConfig* config) {
    scheduler->createMainLoop();
    for (int ii = 0; ii < batch_size; ii++) {
        const long game_index = game_index_base + ii;
        PuctEvaluator* pe = new PuctEvaluator(sm, scheduler, transformer);
        pe->updateConf(&config->puct_config);
        pe->seed(Rng::mix(seed, (uint64_t)game_index, 0));
        evaluators.push_back(pe);
        SelfPlay* sp = new SelfPlay(this, config, pe, sm->initialState(), sm->roleCount(),
                                    identifier + "_" + std::to_string(ii), Rng::mix(seed, (uint64_t)game_index, 1));
        self_plays.push_back(sp);
        scheduler->addRunnable([sp]() { sp->playGamesForever(); });
    }
}

void SelfPlayManager::inflight(long* games, double* engine_s, long* evals) const {
    constexpr int K = OrdinalStats::kOrdinals;
    uint64_t c[K] = {};
    for (int k = 0; k < K; ++k) games[k] = evals[k] = 0;
    for (size_t i = 0; i < self_plays.size(); ++i) {
        const SelfPlay* sp = self_plays[i];
        if (sp->coro == nullptr) continue;
        const int k = std::min(std::max(sp->matchCount(), 1), K) - 1;
        games[k]++;
        const uint64_t now = sp->coro->cycles;   // as of the coroutine's last switch
        if (now > sp->game_c0) c[k] += now - sp->game_c0;
        evals[k] += evaluators[i]->totalEvaluations() - sp->game_e0;
    }
    for (int k = 0; k < K; ++k) engine_s[k] = (double)c[k] / tsc_hz();
}

void SelfPlayManager::poll() {
    stats.polls++;
    stats.evaluations += predict_done_event.pred_count;
    scheduler->poll(&predict_done_event, &ready_event);
}

}  // namespace gz
