// Self-play with lookup_transpositions on (a reference PuctConfig option, off in its self-play
// templates: confs.py:73), under AddressSanitizer: transposed nodes get a second parent, and when
// the first parent's subtree is released (fastApplyMove / releaseNodes) the survivor must not keep
// pointers into it (evaluator.cpp detachEdge).  Driven by a synthetic network (hashed policies /
// values).  Built and run by tests/test_transpositions.py; prints one JSON line of pool counters.
// Usage: transposition_check <game> <batch> <polls> <evals>
#include "../../include/gzero_engine.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static inline unsigned long long mix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline float u01(unsigned long long k) { return (float)(mix64(k) >> 40) * (1.0f / 16777216.0f); }

static gz_puct_config puct(float noise) {
    gz_puct_config c{};
    c.puct_constant = 0.85f; c.puct_constant_root = 0.85f; c.dirichlet_noise_pct = noise;
    c.noise_policy_squash_pct = -1; c.noise_policy_squash_prob = 0.05f; c.choose = 1; c.random_scale = 0.95f;
    c.temperature = 1.0f; c.depth_temperature_start = 2; c.depth_temperature_increment = 0.2f;
    c.depth_temperature_stop = 6; c.depth_temperature_max = 5.0f; c.fpu_prior_discount = 0.25f;
    c.fpu_prior_discount_root = 0.25f; c.top_visits_best_guess_converge_ratio = 0.85f; c.think_time = -1;
    c.converged_visits = 1; c.batch_size = 1; c.use_legals_count_draw = -1;
    c.evaluation_multiplier_to_convergence = 2.0f;
    c.lookup_transpositions = 1;
    return c;
}

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    const char* game = argv[1];
    const int B = atoi(argv[2]), polls = atoi(argv[3]), evals = atoi(argv[4]);
    gz_sm* sm = gz_sm_create(game);
    if (!sm) { std::fprintf(stderr, "%s\n", gz_engine_last_error()); return 1; }
    // breakthrough-style geometry: 2 piece planes, one control plane (the planes' values do not
    // matter to a synthetic network; the transformer only has to be well formed)
    const int side = std::strcmp(game, "breakthroughSmall") == 0 ? 6 : 8;
    const int hw = side * side, P = std::strcmp(game, "breakthroughSmall") == 0 ? 81 : 155;
    int ps[2] = {P, P};
    gz_transformer* t = gz_transformer_create(hw, 2, 1, 1, 2, ps, 2);
    for (int i = 0; i < 2 * hw; ++i) gz_transformer_add_board_base(t, i, hw * (i % 2) + (i / 2));
    gz_transformer_add_control_base(t, 2 * hw, 0, 1.0f);
    gz_transformer_add_control_base(t, 2 * hw + 1, 0, 0.0f);
    const int total = gz_transformer_total_size(t);
    std::vector<float> planes((size_t)B * total), pol0((size_t)B * P), pol1((size_t)B * P), val((size_t)B * 2);
    float* pols[2] = {pol0.data(), pol1.data()};
    gz_pool* pool = gz_pool_create(sm, t, B, "tp", 7, 0, nullptr, planes.data(), pols, val.data());
    if (!pool) { std::fprintf(stderr, "%s\n", gz_engine_last_error()); return 1; }
    gz_selfplay_config conf{};
    conf.oscillate_sampling_pct = 0.25f; conf.temperature_for_policy = 1.0f; conf.puct_config = puct(0.25f);
    conf.evals_per_move = evals; conf.resign0_score_probability = 0.1f; conf.resign0_pct = 0.99f;
    conf.resign1_score_probability = 0.025f; conf.resign1_pct = 0.95f; conf.abort_max_length = -1;
    conf.number_repeat_states_draw = -1; conf.repeat_states_score = 0.5f; conf.run_to_end_pct = 0.01f;
    conf.run_to_end_evals = 32; conf.run_to_end_puct_config = puct(0.15f);
    conf.run_to_end_puct_config.random_scale = 0.75f; conf.run_to_end_early_score = 0.01f;
    conf.run_to_end_minimum_game_depth = 30;
    if (gz_pool_start(pool, &conf) != 0) { std::fprintf(stderr, "%s\n", gz_engine_last_error()); return 1; }
    unsigned long long ctr = 1;
    int rows = gz_pool_poll(pool, 0);
    for (int i = 0; i < polls && rows > 0; ++i) {
        for (int r = 0; r < rows; ++r) {
            for (int k = 0; k < P; ++k) {
                pol0[(size_t)r * P + k] = (0.5f + u01(ctr++)) / P;
                pol1[(size_t)r * P + k] = (0.5f + u01(ctr++)) / P;
            }
            val[r * 2] = u01(ctr++);
            val[r * 2 + 1] = 1 - val[r * 2];
        }
        rows = gz_pool_poll(pool, rows);
        if (rows < 0) { std::fprintf(stderr, "%s\n", gz_engine_last_error()); return 1; }
        if (char* j = gz_pool_fetch_samples(pool)) gz_free(j);
    }
    gz_pool_stats st;
    gz_pool_get_stats(pool, &st);
    std::printf("{\"games_completed\": %ld, \"samples\": %ld, \"transpositions\": %ld, \"evaluations\": %ld}\n",
                st.games_completed, st.samples, st.transpositions, st.evaluations);
    gz_pool_destroy(pool);
    gz_transformer_destroy(t);
    gz_sm_destroy(sm);
    return 0;
}
