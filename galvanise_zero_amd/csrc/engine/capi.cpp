// C-ABI of libgz_engine.so (include/gzero_engine.h).
#include "../../../include/gzero_engine.h"

#include "selfplay.h"
#include "sm.h"
#include "supervisor.h"
#include "transformer.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

using namespace gz;

struct gz_sm { StateMachine* impl; };
struct gz_transformer { GdlBasesTransformer* impl; };
struct gz_supervisor { Supervisor* impl; const StateMachine* sm; const GdlBasesTransformer* t; };
struct gz_player { Player* impl; const StateMachine* sm; };
struct gz_unique_states { UniqueStates* impl; };
struct gz_pool { SelfPlayManager* impl; SelfPlayConfig conf; UniqueStates* own_unique; int num_bases; };

static thread_local std::string g_err;

static int fail(const std::string& m) {
    g_err = m;
    return -1;
}

extern "C" const char* gz_engine_last_error(void) { return g_err.c_str(); }
extern "C" void gz_free(void* p) { std::free(p); }

static char* dup_string(const std::string& s) {
    char* r = (char*)std::malloc(s.size() + 1);
    std::memcpy(r, s.c_str(), s.size() + 1);
    return r;
}

static int copy_out(const std::string& s, char* buf, int buflen) {
    if (buf && buflen > 0) {
        std::strncpy(buf, s.c_str(), buflen - 1);
        buf[buflen - 1] = 0;
    }
    return (int)s.size();
}

// ---- configs ---------------------------------------------------------------------------------
static PuctConfig to_puct(const gz_puct_config& c) {
    PuctConfig p;
    p.verbose = c.verbose != 0;
    p.puct_constant = c.puct_constant;
    p.puct_constant_root = c.puct_constant_root;
    p.dirichlet_noise_pct = c.dirichlet_noise_pct;
    p.noise_policy_squash_pct = c.noise_policy_squash_pct;
    p.noise_policy_squash_prob = c.noise_policy_squash_prob;
    p.choose = c.choose == 1 ? ChooseFn::choose_temperature : ChooseFn::choose_top_visits;
    p.max_dump_depth = c.max_dump_depth;
    p.random_scale = c.random_scale;
    p.temperature = c.temperature;
    p.depth_temperature_start = c.depth_temperature_start;
    p.depth_temperature_increment = c.depth_temperature_increment;
    p.depth_temperature_stop = c.depth_temperature_stop;
    p.depth_temperature_max = c.depth_temperature_max;
    p.fpu_prior_discount = c.fpu_prior_discount;
    p.fpu_prior_discount_root = c.fpu_prior_discount_root;
    p.top_visits_best_guess_converge_ratio = c.top_visits_best_guess_converge_ratio;
    p.think_time = c.think_time;
    p.converged_visits = c.converged_visits;
    p.batch_size = c.batch_size;
    p.use_legals_count_draw = c.use_legals_count_draw;
    p.backup_finalised = c.backup_finalised != 0;
    p.lookup_transpositions = c.lookup_transpositions != 0;
    p.evaluation_multiplier_to_convergence = c.evaluation_multiplier_to_convergence;
    p.spin_yield_playouts = c.spin_yield_playouts;
    return p;
}

static SelfPlayConfig to_selfplay(const gz_selfplay_config& c) {
    SelfPlayConfig s;
    s.oscillate_sampling_pct = c.oscillate_sampling_pct;
    s.temperature_for_policy = c.temperature_for_policy;
    s.puct_config = to_puct(c.puct_config);
    s.evals_per_move = c.evals_per_move;
    s.resign0_score_probability = c.resign0_score_probability;
    s.resign0_pct = c.resign0_pct;
    s.resign1_score_probability = c.resign1_score_probability;
    s.resign1_pct = c.resign1_pct;
    s.abort_max_length = c.abort_max_length;
    s.number_repeat_states_draw = c.number_repeat_states_draw;
    s.repeat_states_score = c.repeat_states_score;
    s.run_to_end_pct = c.run_to_end_pct;
    s.run_to_end_evals = c.run_to_end_evals;
    s.run_to_end_puct_config = to_puct(c.run_to_end_puct_config);
    s.run_to_end_early_score = c.run_to_end_early_score;
    s.run_to_end_minimum_game_depth = c.run_to_end_minimum_game_depth;
    return s;
}

static void to_stats(const PoolStats& s, gz_pool_stats* o) {
    o->games_started = s.games_started;
    o->games_completed = s.games_completed;
    o->games_with_samples = s.games_with_samples;
    o->samples = s.samples;
    o->no_samples = s.no_samples;
    o->dupes = s.dupes;
    o->resigns = s.resigns;
    o->false_positive_resigns0 = s.false_positive_resigns0;
    o->false_positive_resigns1 = s.false_positive_resigns1;
    o->early_run_to_ends = s.early_run_to_ends;
    o->aborts_game_length = s.aborts_game_length;
    o->evaluations = s.evaluations;
    o->polls = s.polls;
    o->completed_game_evals = s.completed_game_evals;
    o->tree_playouts = s.tree_playouts;
    o->transpositions = s.transpositions;
}

// ---- JSON of samples (sampleToDict, supervisor_impl.cpp:75-118) ---------------------------------
static void json_float(std::string& o, float f) {
    char b[32];
    std::snprintf(b, sizeof b, "%.9g", (double)f);
    o += b;
}

static void json_state(std::string& o, const std::vector<uint64_t>& w, int num_bases) {
    o += '[';
    for (int i = 0; i < num_bases; ++i) {
        if (i) o += ',';
        o += bs_get(w.data(), i) ? '1' : '0';
    }
    o += ']';
}

static std::string samples_json(const std::vector<Sample*>& samples, int num_bases) {
    std::string o = "[";
    for (size_t k = 0; k < samples.size(); ++k) {
        const Sample* s = samples[k];
        if (k) o += ',';
        o += "{\"state\":";
        json_state(o, s->state, num_bases);
        o += ",\"prev_states\":[";
        for (size_t i = 0; i < s->prev_states.size(); ++i) {
            if (i) o += ',';
            json_state(o, s->prev_states[i], num_bases);
        }
        o += "],\"policies\":[";
        for (size_t r = 0; r < s->policies.size(); ++r) {
            if (r) o += ',';
            o += '[';
            for (size_t i = 0; i < s->policies[r].size(); ++i) {
                if (i) o += ',';
                o += '[' + std::to_string(s->policies[r][i].first) + ',';
                json_float(o, s->policies[r][i].second);
                o += ']';
            }
            o += ']';
        }
        o += "],\"final_score\":[";
        for (size_t i = 0; i < s->final_score.size(); ++i) {
            if (i) o += ',';
            json_float(o, s->final_score[i]);
        }
        o += "],\"depth\":" + std::to_string(s->depth);
        o += ",\"game_length\":" + std::to_string(s->game_length);
        o += ",\"match_identifier\":\"" + s->match_identifier + "\"";
        o += std::string(",\"has_resigned\":") + (s->has_resigned ? "true" : "false");
        o += std::string(",\"resign_false_positive\":") + (s->resign_false_positive ? "true" : "false");
        o += ",\"starting_sample_depth\":" + std::to_string(s->starting_sample_depth);
        o += ",\"resultant_puct_score\":[";
        for (size_t i = 0; i < s->resultant_puct_score.size(); ++i) {
            if (i) o += ',';
            json_float(o, s->resultant_puct_score[i]);
        }
        o += "],\"resultant_puct_visits\":" + std::to_string(s->resultant_puct_visits) + "}";
    }
    return o + "]";
}

#define GZ_TRY(expr_block)                      \
    try {                                        \
        expr_block                               \
    } catch (const std::exception& e) {          \
        return fail(e.what());                   \
    }

// ---- state machines -----------------------------------------------------------------------------
extern "C" gz_sm* gz_sm_create(const char* game) {
    StateMachine* sm = create_state_machine(game ? game : "");
    if (!sm) {
        fail(std::string("unknown game: ") + (game ? game : "(null)"));
        return nullptr;
    }
    return new gz_sm{sm};
}
extern "C" void gz_sm_destroy(gz_sm* sm) {
    if (sm) {
        delete sm->impl;
        delete sm;
    }
}
extern "C" int gz_sm_role_count(const gz_sm* sm) { return sm->impl->roleCount(); }
extern "C" int gz_sm_num_bases(const gz_sm* sm) { return sm->impl->numBases(); }
extern "C" int gz_sm_num_words(const gz_sm* sm) { return sm->impl->numWords(); }
extern "C" int gz_sm_action_count(const gz_sm* sm, int role) { return sm->impl->actionCount(role); }
extern "C" int gz_sm_base_name(const gz_sm* sm, int i, char* buf, int buflen) {
    return copy_out(sm->impl->baseName(i), buf, buflen);
}
extern "C" int gz_sm_role_name(const gz_sm* sm, int role, char* buf, int buflen) {
    return copy_out(sm->impl->roleName(role), buf, buflen);
}
extern "C" int gz_sm_legal_to_move(const gz_sm* sm, int role, int action, char* buf, int buflen) {
    return copy_out(sm->impl->legalToMove(role, action), buf, buflen);
}
extern "C" int gz_sm_initial_state(const gz_sm* sm, uint64_t* out) {
    std::memcpy(out, sm->impl->initialState(), sizeof(uint64_t) * sm->impl->numWords());
    return 0;
}
extern "C" int gz_sm_update_bases(gz_sm* sm, const uint64_t* state) {
    sm->impl->updateBases(state);
    return 0;
}
extern "C" int gz_sm_legal_count(const gz_sm* sm, int role) { return sm->impl->legalCount(role); }
extern "C" int gz_sm_legal(const gz_sm* sm, int role, int i) { return sm->impl->legal(role, i); }
extern "C" int gz_sm_is_terminal(const gz_sm* sm) { return sm->impl->isTerminal() ? 1 : 0; }
extern "C" int gz_sm_goal_value(const gz_sm* sm, int role) { return sm->impl->goalValue(role); }
extern "C" int gz_sm_next_state(gz_sm* sm, const int* joint_move, uint64_t* out) {
    JointMove m{};
    for (int r = 0; r < sm->impl->roleCount(); ++r) m.set(r, joint_move[r]);
    sm->impl->nextState(m, out);
    return 0;
}

// ---- transformer ------------------------------------------------------------------------------
extern "C" gz_transformer* gz_transformer_create(int channel_size, int channels_per_state, int num_control_channels,
                                                 int num_prev_states, int num_rewards, const int* policy_sizes,
                                                 int num_policies) {
    if (num_policies < 1 || num_policies > kMaxRoles || num_rewards < 1 || num_rewards > 4) {
        fail("bad transformer arguments");
        return nullptr;
    }
    std::vector<int> ps(policy_sizes, policy_sizes + num_policies);
    return new gz_transformer{new GdlBasesTransformer(channel_size, channels_per_state, num_control_channels,
                                                      num_prev_states, num_rewards, ps)};
}
extern "C" void gz_transformer_destroy(gz_transformer* t) {
    if (t) {
        delete t->impl;
        delete t;
    }
}
extern "C" int gz_transformer_add_board_base(gz_transformer* t, int base_indx, int buf_incr) {
    t->impl->addBoardBase(base_indx, buf_incr);
    return 0;
}
extern "C" int gz_transformer_add_control_base(gz_transformer* t, int base_indx, int channel_id, float value) {
    t->impl->addControlBase(base_indx, channel_id, value);
    return 0;
}
extern "C" int gz_transformer_total_size(const gz_transformer* t) { return t->impl->totalSize(); }
extern "C" int gz_transformer_to_channels(const gz_transformer* t, const uint64_t* state,
                                          const uint64_t* const* prev_states, int num_prev, float* out) {
    std::vector<const uint64_t*> prev(prev_states, prev_states + num_prev);
    t->impl->toChannels(state, prev, out);
    return 0;
}

// ---- supervisor -------------------------------------------------------------------------------
extern "C" gz_supervisor* gz_supervisor_create(const gz_sm* sm, const gz_transformer* t, int batch_size,
                                               const char* identifier, uint64_t seed, int per_pool_unique_states) {
    if (!sm || !t || batch_size < 1) {
        fail("bad supervisor arguments");
        return nullptr;
    }
    return new gz_supervisor{new Supervisor(sm->impl, t->impl, batch_size, identifier ? identifier : "", seed,
                                            per_pool_unique_states != 0),
                             sm->impl, t->impl};
}
extern "C" void gz_supervisor_destroy(gz_supervisor* s) {
    if (s) {
        delete s->impl;
        delete s;
        node_cache_flush();
    }
}
extern "C" int gz_supervisor_start_self_play(gz_supervisor* s, int num_workers, const gz_selfplay_config* conf) {
    if (!s || !conf) return fail("null argument");
    GZ_TRY({
        SelfPlayConfig c = to_selfplay(*conf);
        if (num_workers <= 0) s->impl->createInline(&c);
        else
            for (int i = 0; i < num_workers; ++i) s->impl->createWorkers(&c);
    })
    return 0;
}
extern "C" int gz_supervisor_cancel(gz_supervisor* s) {
    if (!s) return fail("null supervisor");
    s->impl->cancel();
    return 0;
}
extern "C" float* gz_supervisor_poll(gz_supervisor* s, int predict_count, float* const* arrays, int num_arrays,
                                     int* buf_count) {
    *buf_count = -1;
    const int expect = s->t->getNumberPolicies() + 1;
    if (num_arrays != expect) {
        fail("poll expects " + std::to_string(expect) + " arrays");
        return nullptr;
    }
    try {
        std::vector<float*> data(arrays, arrays + num_arrays);
        const ReadyEvent* ev = s->impl->poll(predict_count, data);
        *buf_count = ev->buf_count;
        return ev->buf_count ? ev->channel_buf : nullptr;
    } catch (const std::exception& e) {
        fail(e.what());
        return nullptr;
    }
}
extern "C" char* gz_supervisor_fetch_samples(gz_supervisor* s) {
    std::vector<Sample*> samples = s->impl->getSamples();
    if (samples.empty()) return nullptr;
    std::string j = samples_json(samples, s->sm->numBases());
    for (Sample* x : samples) delete x;
    return dup_string(j);
}
extern "C" int gz_supervisor_add_unique_state(gz_supervisor* s, const uint64_t* state) {
    s->impl->addUniqueState(state);
    return 0;
}
extern "C" int gz_supervisor_clear_unique_states(gz_supervisor* s) {
    s->impl->clearUniqueStates();
    return 0;
}
extern "C" int gz_supervisor_set_sample_interval(gz_supervisor* s, int polls) {
    s->impl->setSampleInterval(polls);
    return 0;
}
extern "C" int gz_supervisor_stats(gz_supervisor* s, gz_pool_stats* out) {
    to_stats(s->impl->stats(), out);
    return 0;
}

// ---- player -----------------------------------------------------------------------------------
extern "C" gz_player* gz_player_create(const gz_sm* sm, const gz_transformer* t, const gz_puct_config* conf,
                                       uint64_t seed) {
    if (!sm || !t || !conf) {
        fail("null argument");
        return nullptr;
    }
    return new gz_player{new Player(sm->impl, t->impl, to_puct(*conf), seed), sm->impl};
}
extern "C" void gz_player_destroy(gz_player* p) {
    if (p) {
        delete p->impl;
        delete p;
        node_cache_flush();
    }
}
extern "C" int gz_player_reset(gz_player* p, int game_depth) {
    p->impl->puctPlayerReset(game_depth);
    return 0;
}
extern "C" int gz_player_apply_move(gz_player* p, const int* joint_move) {
    JointMove m{};
    for (int r = 0; r < p->sm->roleCount(); ++r) m.set(r, joint_move[r]);
    p->impl->puctApplyMove(m);
    return 0;
}
extern "C" int gz_player_move(gz_player* p, const uint64_t* state, int iterations, double end_time) {
    p->impl->puctPlayerMove(state, iterations, end_time);
    return 0;
}
extern "C" int gz_player_get_move(gz_player* p, int lead_role_index, int* legal, float* probability, int* node_count) {
    auto t = p->impl->puctPlayerGetMove(lead_role_index);
    *legal = std::get<0>(t);
    *probability = std::get<1>(t);
    *node_count = std::get<2>(t);
    return 0;
}
extern "C" int gz_player_update_config(gz_player* p, double think_time, int converged_visits, int verbose) {
    p->impl->updateConfig((float)think_time, converged_visits, verbose != 0);
    return 0;
}
extern "C" int gz_player_balance_moves(gz_player* p, int max_count) {
    p->impl->balanceNode(max_count);
    return 0;
}
extern "C" char* gz_player_tree_debug(gz_player* p, int max_count) {
    std::vector<PuctNodeDebug> infos = p->impl->treeDebugInfo(max_count);
    std::string o = "[";
    for (size_t i = 0; i < infos.size(); ++i) {
        if (i) o += ',';
        o += "{\"lead_role_index\":" + std::to_string(infos[i].lead_role_index);
        o += ",\"move_index\":" + std::to_string(infos[i].move_index) + ",\"score\":";
        json_float(o, infos[i].score);
        o += ",\"variation\":[";
        for (size_t k = 0; k < infos[i].variation.size(); ++k) {
            if (k) o += ',';
            o += "[" + std::to_string(infos[i].variation[k].first) + "," + std::to_string(infos[i].variation[k].second) + "]";
        }
        o += "]}";
    }
    return dup_string(o + "]");
}
extern "C" float* gz_player_poll(gz_player* p, int predict_count, float* const* arrays, int num_arrays, int* buf_count) {
    *buf_count = -1;
    try {
        std::vector<float*> data(arrays, arrays + num_arrays);
        const ReadyEvent* ev = p->impl->poll(predict_count, data);
        *buf_count = ev->buf_count;
        return ev->buf_count ? ev->channel_buf : nullptr;
    } catch (const std::exception& e) {
        fail(e.what());
        return nullptr;
    }
}
extern "C" int gz_player_root_children(gz_player* p, int* moves, uint32_t* traversals, float* policy_probs, int cap) {
    const PuctNode* root = p->impl->getEvaluator()->getRootNode();
    if (!root) return 0;
    const int n = std::min((int)root->num_children, cap);
    const int lead = root->lead_role_index < 0 ? 0 : root->lead_role_index;
    for (int i = 0; i < n; ++i) {
        const PuctNodeChild* c = root->getNodeChild(0, i);
        if (moves) moves[i] = root->cold()[i].move.get(lead);
        if (traversals) traversals[i] = c->traversals;
        if (policy_probs) policy_probs[i] = c->policy_prob;
    }
    return root->num_children;
}

// ---- pools --------------------------------------------------------------------------------------
extern "C" gz_unique_states* gz_unique_states_create(const gz_sm* sm, const gz_transformer* t, int max_num_dupes) {
    return new gz_unique_states{new UniqueStates(t->impl->createHashMask(sm->impl->numBases()), max_num_dupes)};
}
extern "C" void gz_unique_states_destroy(gz_unique_states* u) {
    if (u) {
        delete u->impl;
        delete u;
    }
}
extern "C" int gz_unique_states_clear(gz_unique_states* u) {
    if (!u) return fail("null unique states");
    u->impl->clear();
    return 0;
}
extern "C" gz_pool* gz_pool_create(const gz_sm* sm, const gz_transformer* t, int batch_size, const char* identifier,
                                   uint64_t seed, long game_index_base, gz_unique_states* unique_states,
                                   float* planes_buf, float* const* policy_bufs, float* value_buf) {
    if (!sm || !t || batch_size < 1) {
        fail("bad pool arguments");
        return nullptr;
    }
    gz_pool* p = new gz_pool;
    p->own_unique = nullptr;
    UniqueStates* u;
    if (unique_states) {
        u = unique_states->impl;
    } else {
        u = p->own_unique = new UniqueStates(t->impl->createHashMask(sm->impl->numBases()), 1000);
    }
    p->num_bases = sm->impl->numBases();
    p->impl = new SelfPlayManager(sm->impl, t->impl, batch_size, u, identifier ? identifier : "pool", seed,
                                  game_index_base, planes_buf, policy_bufs, value_buf);
    return p;
}
extern "C" void gz_pool_destroy(gz_pool* p) {
    if (p) {
        delete p->impl;
        delete p->own_unique;
        delete p;
        node_cache_flush();   // the trees were freed onto this thread's lists
    }
}
extern "C" int gz_pool_start(gz_pool* p, const gz_selfplay_config* conf) {
    p->conf = to_selfplay(*conf);
    p->impl->startSelfPlayers(&p->conf);
    return 0;
}
extern "C" int gz_pool_cancel(gz_pool* p) {
    if (!p) return fail("null pool");
    p->impl->cancel();
    return 0;
}
extern "C" int gz_pool_poll(gz_pool* p, int pred_count) {
    p->impl->getPredictDoneEvent()->pred_count = pred_count;
    p->impl->poll();
    const int ts = p->impl->getTransformer()->totalSize();
    return p->impl->getReadyEvent()->buf_count / ts;
}
// the pool's own duplicate filter (pools created without a shared one); supervisor_impl.cpp:138-144
extern "C" int gz_pool_clear_unique_states(gz_pool* p) {
    if (!p) return fail("null pool");
    if (p->own_unique) p->own_unique->clear();
    return 0;
}
extern "C" int gz_pool_get_stats(gz_pool* p, gz_pool_stats* out) {
    PoolStats s = p->impl->getStats();
    s.tree_playouts = p->impl->treePlayouts();
    s.transpositions = p->impl->transpositions();
    to_stats(s, out);
    return 0;
}
extern "C" char* gz_pool_fetch_samples(gz_pool* p) {
    std::vector<Sample*>& s = p->impl->getSamples();
    if (s.empty()) return nullptr;
    std::string j = samples_json(s, p->num_bases);
    for (Sample* x : s) delete x;
    s.clear();
    return dup_string(j);
}
extern "C" char* gz_pool_fetch_samples_n(gz_pool* p, long* count) {
    std::vector<Sample*>& s = p->impl->getSamples();
    *count = (long)s.size();
    if (s.empty()) return nullptr;
    std::string j = samples_json(s, p->num_bases);
    for (Sample* x : s) delete x;
    s.clear();
    return dup_string(j);
}
static_assert(GZ_ORDINALS == OrdinalStats::kOrdinals && GZ_COST_HIST == OrdinalStats::kHist, "ordinal stats layout");
extern "C" int gz_pool_add_ordinal_stats(gz_pool* p, gz_ordinal_stats* out) {
    if (!p || !out) return fail("null argument");
    const OrdinalStats& o = p->impl->getStats().ord;
    const double hz = tsc_hz();
    for (int k = 0; k < GZ_ORDINALS; ++k) {
        out->games[k] += o.games[k];
        out->evals[k] += o.evals[k];
        out->tree_playouts[k] += o.tree_playouts[k];
        out->moves[k] += o.moves[k];
        out->spin_epochs[k] += o.spin_epochs[k];
        out->engine_s[k] += (double)o.cycles[k] / hz;
    }
    for (int k = 0; k < GZ_COST_HIST; ++k) out->cost_hist[k] += o.cost_hist[k];
    long g[GZ_ORDINALS], e[GZ_ORDINALS];
    double s[GZ_ORDINALS];
    p->impl->inflight(g, s, e);
    for (int k = 0; k < GZ_ORDINALS; ++k) {
        out->inflight_games += g[k];
        out->inflight_engine_s += s[k];
        out->inflight_evals += e[k];
        out->inflight_games_ord[k] += g[k];
        out->inflight_engine_s_ord[k] += s[k];
        out->inflight_evals_ord[k] += e[k];
    }
    return 0;
}
extern "C" int gz_engine_set_verify_fastpath(int on) {
    const bool prev = get_verify_fastpath();
    set_verify_fastpath(on != 0);
    return prev ? 1 : 0;
}
extern "C" long gz_engine_verified_decisions(void) { return verified_decisions(); }
#ifndef GZ_BUILD_PGO
#define GZ_BUILD_PGO "unknown"
#endif
#ifndef GZ_BUILD_MARCH
#define GZ_BUILD_MARCH "unknown"
#endif
extern "C" const char* gz_engine_build_info(void) { return "pgo=" GZ_BUILD_PGO " march=" GZ_BUILD_MARCH; }
extern "C" long gz_pool_take_sample_count(gz_pool* p) {
    std::vector<Sample*>& s = p->impl->getSamples();
    const long n = (long)s.size();
    for (Sample* x : s) delete x;
    s.clear();
    return n;
}
