/* gzero_engine.h -- C-ABI of the native self-play engine (libgz_engine.so).
 *
 * Replaces the CPython-2 extension module `ggpzero_interface` (reference
 * src/cpp/ggpzero_interface.cpp:65-95, src/cpp/pyobjects/ (common, supervisor_impl, player_impl)) and the ggplib state-machine
 * pointer it is handed (cppinterface.py:12-16).  Python binds it with ctypes
 * (galvanise_zero_amd/_native.py); INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions: plain pointers and sizes; functions returning int return >= 0 on success and -1 on
 * error (gz_engine_last_error() holds the message, thread-local).  Internal invariant violations
 * abort, as the reference's ASSERT does.
 */
#ifndef GZERO_ENGINE_H
#define GZERO_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gz_sm gz_sm;
typedef struct gz_transformer gz_transformer;
typedef struct gz_supervisor gz_supervisor;
typedef struct gz_player gz_player;
typedef struct gz_pool gz_pool;
typedef struct gz_unique_states gz_unique_states;

/* PuctConfig (src/cpp/puct/config.h:11-53), filled from confs.PUCTEvaluatorConfig
 * (src/ggpzero/defs/confs.py:9-73) by createPuctConfig (src/cpp/pyobjects/common.cpp:48-113).
 * choose: 0 = choose_top_visits, 1 = choose_temperature. */
typedef struct gz_puct_config {
    int verbose;
    float puct_constant;
    float puct_constant_root;
    float dirichlet_noise_pct;
    float noise_policy_squash_pct;
    float noise_policy_squash_prob;
    int choose;
    int max_dump_depth;
    float random_scale;
    float temperature;
    int depth_temperature_start;
    float depth_temperature_increment;
    int depth_temperature_stop;
    float depth_temperature_max;
    float fpu_prior_discount;
    float fpu_prior_discount_root;
    float top_visits_best_guess_converge_ratio;
    float think_time;
    int converged_visits;
    int batch_size;
    int use_legals_count_draw;
    int backup_finalised;
    int lookup_transpositions;
    float evaluation_multiplier_to_convergence;
    int spin_yield_playouts;     /* build extension, 0 = reference behaviour (engine/config.h) */
} gz_puct_config;

/* SelfPlayConfig (src/cpp/selfplay.h:19-41), filled from confs.SelfPlayConfig (confs.py:93-123)
 * by createSelfPlayConfig (common.cpp:116-158); missing keys keep their defaults. */
typedef struct gz_selfplay_config {
    float oscillate_sampling_pct;
    float temperature_for_policy;
    gz_puct_config puct_config;
    int evals_per_move;
    float resign0_score_probability;
    float resign0_pct;
    float resign1_score_probability;
    float resign1_pct;
    int abort_max_length;
    int number_repeat_states_draw;
    float repeat_states_score;
    float run_to_end_pct;
    int run_to_end_evals;
    gz_puct_config run_to_end_puct_config;
    float run_to_end_early_score;
    int run_to_end_minimum_game_depth;
} gz_selfplay_config;

/* Counters of SelfPlayManager::reportAndResetStats (selfplaymanager.cpp:161-200) plus throughput
 * counters (games, NN rows). */
typedef struct gz_pool_stats {
    long games_started;
    long games_completed;
    long games_with_samples;
    long samples;
    long no_samples;
    long dupes;
    long resigns;
    long false_positive_resigns0;
    long false_positive_resigns1;
    long early_run_to_ends;
    long aborts_game_length;
    long evaluations;
    long polls;
    long completed_game_evals;   /* NN evaluations consumed by the completed games */
    long tree_playouts;          /* tree playouts (treePlayout calls), NN-free ones included */
    long transpositions;         /* edges attached to an existing node (lookup_transpositions) */
} gz_pool_stats;

/* Per-game cost by the game's ordinal within its slot (a slot = one SelfPlay of a pool; its 1st,
 * 2nd, ... game; the last bucket holds every later game), for the steady-state analysis (DESIGN.md
 * section 6).  Build diagnostics: the reference has no counterpart. */
#define GZ_ORDINALS 8
#define GZ_COST_HIST 32
typedef struct gz_ordinal_stats {
    long games[GZ_ORDINALS];          /* completed games */
    long evals[GZ_ORDINALS];          /* NN evaluations they used */
    long tree_playouts[GZ_ORDINALS];  /* tree playouts (NN-free ones included) */
    long moves[GZ_ORDINALS];          /* moves played */
    long spin_epochs[GZ_ORDINALS];    /* root spin epochs built (engine fast path) */
    double engine_s[GZ_ORDINALS];     /* engine-thread seconds inside the games' coroutines (TSC) */
    long cost_hist[GZ_COST_HIST];     /* completed games by engine ms: bucket k = [2^(k-1), 2^k) ms */
    long inflight_games;              /* games in progress at the snapshot */
    double inflight_engine_s;         /* engine seconds they have used so far */
    long inflight_evals;              /* evaluations they have used so far */
    long inflight_games_ord[GZ_ORDINALS];      /* the same by the in-progress game's ordinal */
    double inflight_engine_s_ord[GZ_ORDINALS];
    long inflight_evals_ord[GZ_ORDINALS];
} gz_ordinal_stats;

const char* gz_engine_last_error(void);
void gz_free(void* p);                         /* frees strings returned by this library */

/* ---- state machines (ggplib StateMachineInterface stand-in) -------------------------------- */
gz_sm* gz_sm_create(const char* game);         /* "breakthrough", "breakthroughSmall", ... */
void gz_sm_destroy(gz_sm* sm);
int gz_sm_role_count(const gz_sm* sm);
int gz_sm_num_bases(const gz_sm* sm);
int gz_sm_num_words(const gz_sm* sm);          /* uint64 words per base state */
int gz_sm_action_count(const gz_sm* sm, int role);
int gz_sm_base_name(const gz_sm* sm, int index, char* buf, int buflen);
int gz_sm_role_name(const gz_sm* sm, int role, char* buf, int buflen);
int gz_sm_legal_to_move(const gz_sm* sm, int role, int action, char* buf, int buflen);
int gz_sm_initial_state(const gz_sm* sm, uint64_t* out);
int gz_sm_update_bases(gz_sm* sm, const uint64_t* state);
int gz_sm_legal_count(const gz_sm* sm, int role);
int gz_sm_legal(const gz_sm* sm, int role, int i);
int gz_sm_is_terminal(const gz_sm* sm);
int gz_sm_goal_value(const gz_sm* sm, int role);
int gz_sm_next_state(gz_sm* sm, const int* joint_move, uint64_t* out);

/* ---- GdlBasesTransformer (gi_GdlBasesTransformer, gdltransformer_impl.cpp:186-219) ---------- */
gz_transformer* gz_transformer_create(int channel_size, int channels_per_state, int num_control_channels,
                                      int num_prev_states, int num_rewards, const int* policy_sizes,
                                      int num_policies);
void gz_transformer_destroy(gz_transformer* t);
int gz_transformer_add_board_base(gz_transformer* t, int base_indx, int buf_incr);
int gz_transformer_add_control_base(gz_transformer* t, int base_indx, int channel_id, float value);
int gz_transformer_total_size(const gz_transformer* t);
int gz_transformer_to_channels(const gz_transformer* t, const uint64_t* state, const uint64_t* const* prev_states,
                               int num_prev, float* out);

/* ---- Supervisor (gi_Supervisor + Supervisor_methods, supervisor_impl.cpp:150-237) ----------- */
/* seed: global RNG seed; per_pool_unique_states: 1 = deterministic (each pool its own duplicate
 * filter), 0 = reference behaviour (one filter shared by every pool, supervisor.cpp:31). */
gz_supervisor* gz_supervisor_create(const gz_sm* sm, const gz_transformer* t, int batch_size,
                                    const char* identifier, uint64_t seed, int per_pool_unique_states);
void gz_supervisor_destroy(gz_supervisor* s);
int gz_supervisor_start_self_play(gz_supervisor* s, int num_workers, const gz_selfplay_config* conf);
/* doPoll (common.cpp:161-218): arrays = R policy buffers [predict_count*P_r] then values
 * [predict_count*V]; returns the engine-owned planes buffer and *buf_count floats (valid until the
 * next poll); NULL with *buf_count 0 when finished, NULL with *buf_count -1 on error. */
float* gz_supervisor_poll(gz_supervisor* s, int predict_count, float* const* arrays, int num_arrays, int* buf_count);
/* Bounded teardown from any thread (build extension; the reference ends its workers with the
 * process): every pool is cancelled (gz_pool_cancel) and gz_supervisor_poll -- one in progress
 * included -- returns NULL with *buf_count 0 from then on. */
int gz_supervisor_cancel(gz_supervisor* s);
/* fetch_samples: JSON list of Sample dicts (datadesc.py:8-38 / sampleToDict supervisor_impl.cpp:75-118)
 * or NULL when there are none; free with gz_free. */
char* gz_supervisor_fetch_samples(gz_supervisor* s);
int gz_supervisor_add_unique_state(gz_supervisor* s, const uint64_t* state);
int gz_supervisor_clear_unique_states(gz_supervisor* s);
int gz_supervisor_stats(gz_supervisor* s, gz_pool_stats* out);
/* polls between moving pool samples to the supervisor (reference fixed at 1024) */
int gz_supervisor_set_sample_interval(gz_supervisor* s, int polls);

/* ---- Player (gi_Player + Player_methods, player_impl.cpp:116-201) --------------------------- */
gz_player* gz_player_create(const gz_sm* sm, const gz_transformer* t, const gz_puct_config* conf, uint64_t seed);
void gz_player_destroy(gz_player* p);
int gz_player_reset(gz_player* p, int game_depth);
int gz_player_apply_move(gz_player* p, const int* joint_move);
int gz_player_move(gz_player* p, const uint64_t* state, int iterations, double end_time);
int gz_player_get_move(gz_player* p, int lead_role_index, int* legal, float* probability, int* node_count);
int gz_player_update_config(gz_player* p, double think_time, int converged_visits, int verbose);
int gz_player_balance_moves(gz_player* p, int max_count);
char* gz_player_tree_debug(gz_player* p, int max_count);    /* JSON; free with gz_free */
float* gz_player_poll(gz_player* p, int predict_count, float* const* arrays, int num_arrays, int* buf_count);
/* root children after a move: counts = traversals, probs = policy_prob, moves = lead-role action */
int gz_player_root_children(gz_player* p, int* moves, uint32_t* traversals, float* policy_probs, int cap);

/* ---- game pools for the native GPU driver (one SelfPlayManager each) ------------------------ */
gz_unique_states* gz_unique_states_create(const gz_sm* sm, const gz_transformer* t, int max_num_dupes);
void gz_unique_states_destroy(gz_unique_states* u);
/* UniqueStates::clear (clear_unique_states, supervisor_impl.cpp:138-144): a new generation starts
 * with an empty duplicate filter (worker.py:160). */
int gz_unique_states_clear(gz_unique_states* u);
/* planes_buf [batch*total_size], policy_bufs[r] [batch*P_r], value_buf [batch*V] are caller-owned
 * (e.g. pinned host memory); predictions must be written there before gz_pool_poll(pred_count). */
gz_pool* gz_pool_create(const gz_sm* sm, const gz_transformer* t, int batch_size, const char* identifier,
                        uint64_t seed, long game_index_base, gz_unique_states* unique_states,
                        float* planes_buf, float* const* policy_bufs, float* value_buf);
void gz_pool_destroy(gz_pool* p);
int gz_pool_start(gz_pool* p, const gz_selfplay_config* conf);
int gz_pool_poll(gz_pool* p, int pred_count);   /* returns rows of planes now in planes_buf */
/* Teardown, callable from any thread while another thread is inside gz_pool_poll: the poll in
 * progress returns 0 rows at the pool's next coroutine switch (a game's next evaluation or yield;
 * a game that spins without evaluations yields after every playout once cancelled), and so does
 * every later poll.  The games in progress are abandoned (freed by gz_pool_destroy); samples
 * already emitted are unchanged.  The reference tears its workers down with the process
 * (supervisor.cpp:36); a runner hosting live rolls needs a bounded stop instead. */
int gz_pool_cancel(gz_pool* p);
int gz_pool_get_stats(gz_pool* p, gz_pool_stats* out);
/* clears the pool's own duplicate filter (no-op for a pool created with a shared one) */
int gz_pool_clear_unique_states(gz_pool* p);
char* gz_pool_fetch_samples(gz_pool* p);          /* JSON or NULL; free with gz_free */
long gz_pool_take_sample_count(gz_pool* p);       /* drops queued samples, returns how many */
/* adds the pool's per-ordinal counters into *out (zero it first to read one pool) */
int gz_pool_add_ordinal_stats(gz_pool* p, gz_ordinal_stats* out);

/* ---- run-time verification of the engine's fast paths (build diagnostics) -------------------- */
/* on = 1: every sort-free selection, spin playout and register spin run is re-checked against the
 * literal reference path, aborting on a difference (what GZ_VERIFY_FASTPATH=1 sets at load);
 * process-wide, takes effect at the next decision; returns the previous setting. */
int gz_engine_set_verify_fastpath(int on);
/* fast-path decisions re-checked so far (process-wide) */
long gz_engine_verified_decisions(void);
char* gz_pool_fetch_samples_n(gz_pool* p, long* count);  /* as fetch_samples, *count = records */

/* How this library was built (static string): "pgo=<use|none|stale|gen> march=<...>" -- use: gcc
 * profiles recorded on these exact sources (csrc/pgo/sources.sha256); stale: profiles present but
 * recorded on other sources, so not used.  Reported in the bench line. */
const char* gz_engine_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* GZERO_ENGINE_H */
