// Search / self-play configuration.  Field-for-field restatement of PuctConfig
// (reference src/cpp/puct/config.h:11-53) and SelfPlayConfig (src/cpp/selfplay.h:19-41); the
// Python side fills them from the same attrs dicts the reference passes (confs.py:9-123,
// common.cpp:48-158).
#pragma once

namespace gz {

enum class ChooseFn { choose_top_visits = 0, choose_temperature = 1 };

struct PuctConfig {
    bool verbose = false;
    float puct_constant = 0.85f;
    float puct_constant_root = 2.5f;
    float dirichlet_noise_pct = 0.25f;
    float noise_policy_squash_pct = -1.0f;
    float noise_policy_squash_prob = 0.05f;
    ChooseFn choose = ChooseFn::choose_top_visits;
    int max_dump_depth = 2;
    float random_scale = 0.5f;
    float temperature = 1.0f;
    int depth_temperature_start = 5;
    float depth_temperature_increment = 0.5f;
    int depth_temperature_stop = 10;
    float depth_temperature_max = 5.0f;
    float fpu_prior_discount = 0.25f;
    float fpu_prior_discount_root = 0.25f;
    float top_visits_best_guess_converge_ratio = 0.8f;
    float think_time = 10.0f;
    int converged_visits = 5000;
    int batch_size = 32;
    int use_legals_count_draw = -1;
    bool backup_finalised = false;
    bool lookup_transpositions = false;
    float evaluation_multiplier_to_convergence = 1.0f;
    // Build extension (not in the reference config, default off = reference behaviour): after this
    // many consecutive tree playouts without a new NN evaluation, playoutMain yields to the
    // scheduler, as the reference's playoutWorker already does for its tight loop
    // (evaluator.cpp:725-730).  A game stuck proving a lost root (every playout ends on a terminal
    // node, evaluator.cpp:794-841 has no break for it) then no longer stalls its pool mates; the
    // game's own search is unchanged (batch-invariant NN, per-game RNG).
    int spin_yield_playouts = 0;
};

struct SelfPlayConfig {
    float oscillate_sampling_pct = 0.25f;
    float temperature_for_policy = 1.0f;
    PuctConfig puct_config;
    int evals_per_move = 800;
    float resign0_score_probability = 0.9f;
    float resign0_pct = 0.5f;
    float resign1_score_probability = 0.975f;
    float resign1_pct = 0.1f;
    int abort_max_length = -1;
    int number_repeat_states_draw = -1;
    float repeat_states_score = 0.5f;
    float run_to_end_pct = 0.2f;
    int run_to_end_evals = 42;
    PuctConfig run_to_end_puct_config;
    float run_to_end_early_score = 0.01f;
    int run_to_end_minimum_game_depth = 30;
};

}  // namespace gz
