// Host-only engine throughput probe: T threads x one pool of breakthrough self-play each, driven by a
// synthetic network (random policy / value), no GPU.  Reports microseconds of tree work per leaf.
// Usage: engine_bench [batch] [polls] [evals] [threads] [spin_yield]
//   g++ -O2 -std=c++17 -ffp-contract=off -march=x86-64-v3 tools/engine_bench.cpp galvanise_zero_amd/csrc/engine/*.cpp -o /tmp/engine_bench -pthread
#include "../include/gzero_engine.h"

#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <vector>

// synthetic network: a counter hash (splitmix64) instead of a std::mt19937 stream, so the probe's
// own cost stays small next to the engine's
static inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline float u01(uint64_t k) { return (float)(mix64(k) >> 40) * (1.0f / 16777216.0f); }

static gz_puct_config base_puct(float noise) {
    gz_puct_config c{};
    c.puct_constant = 0.85f; c.puct_constant_root = 0.85f; c.dirichlet_noise_pct = noise;
    c.noise_policy_squash_pct = -1; c.noise_policy_squash_prob = 0.05f; c.choose = 1; c.random_scale = 0.95f;
    c.temperature = 1.0f; c.depth_temperature_start = 2; c.depth_temperature_increment = 0.2f;
    c.depth_temperature_stop = 6; c.depth_temperature_max = 5.0f; c.fpu_prior_discount = 0.25f;
    c.fpu_prior_discount_root = 0.25f; c.top_visits_best_guess_converge_ratio = 0.85f; c.think_time = -1;
    c.converged_visits = 1; c.batch_size = 1; c.use_legals_count_draw = -1;
    c.evaluation_multiplier_to_convergence = 2.0f;
    return c;
}

static void run(int tid, int B, int polls, int evals, int spin) {
    gz_sm* sm = gz_sm_create("breakthrough");
    int ps[2] = {155, 155};
    gz_transformer* t = gz_transformer_create(64, 2, 1, 1, 2, ps, 2);
    for (int i = 0; i < 128; ++i) {
        const int cell = i / 2, p = i % 2, x = cell / 8, y = cell % 8;
        gz_transformer_add_board_base(t, i, 64 * p + y * 8 + x);
    }
    gz_transformer_add_control_base(t, 128, 0, 1.0f);
    gz_transformer_add_control_base(t, 129, 0, 0.0f);
    std::vector<float> planes((size_t)B * 320), pol0((size_t)B * 155), pol1((size_t)B * 155), val((size_t)B * 2);
    float* pols[2] = {pol0.data(), pol1.data()};
    gz_pool* pool = gz_pool_create(sm, t, B, "bench", 1, (long)tid * B, nullptr, planes.data(), pols, val.data());
    gz_selfplay_config conf{};
    conf.oscillate_sampling_pct = 0.25f; conf.temperature_for_policy = 1.0f; conf.puct_config = base_puct(0.25f);
    conf.evals_per_move = evals; conf.resign0_score_probability = 0.1f; conf.resign0_pct = 0.99f;
    conf.resign1_score_probability = 0.025f; conf.resign1_pct = 0.95f; conf.abort_max_length = -1;
    conf.number_repeat_states_draw = -1; conf.repeat_states_score = 0.5f; conf.run_to_end_pct = 0.01f;
    conf.run_to_end_evals = 32; conf.run_to_end_puct_config = base_puct(0.15f);
    conf.run_to_end_puct_config.random_scale = 0.75f; conf.run_to_end_early_score = 0.01f;
    conf.run_to_end_minimum_game_depth = 30;
    conf.puct_config.spin_yield_playouts = spin;
    conf.run_to_end_puct_config.spin_yield_playouts = spin;
    gz_pool_start(pool, &conf);
    uint64_t ctr = (uint64_t)(tid + 1) << 40;
    int rows = gz_pool_poll(pool, 0);
    long leaves = 0;
    long tp_prev = 0;
    double tt = 0, worst = 0, win_t = 0;
    long win_l = 0;
    for (int i = 0; i < polls; ++i) {
        for (int r = 0; r < rows; ++r) {   // roughly uniform policies, uniform value
            for (int k = 0; k < 155; ++k) {
                pol0[r * 155 + k] = (0.5f + u01(ctr++)) * (1.0f / 155);
                pol1[r * 155 + k] = (0.5f + u01(ctr++)) * (1.0f / 155);
            }
            val[r * 2] = u01(ctr++); val[r * 2 + 1] = 1 - val[r * 2];
        }
        auto a = std::chrono::steady_clock::now();
        const int done = rows;
        rows = gz_pool_poll(pool, done);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
        if (i >= 50) { tt += dt; leaves += done; if (dt > worst) worst = dt; }
        win_t += dt;
        win_l += done;
        if (tid == 0 && (i + 1) % 2000 == 0) {
            gz_pool_stats ws;
            gz_pool_get_stats(pool, &ws);
            std::printf("thread 0 polls %6d: window %.2f us/leaf, %.1f tree playouts/leaf, games %ld\n", i + 1,
                        win_t / win_l * 1e6, (double)(ws.tree_playouts - tp_prev) / win_l, ws.games_completed);
            tp_prev = ws.tree_playouts;
            std::fflush(stdout);
            win_t = 0;
            win_l = 0;
        }
    }
    gz_pool_stats st;
    gz_pool_get_stats(pool, &st);
    std::printf("thread %d B=%d polls=%d: %.3f us/leaf, worst poll %.1f ms, games completed %ld, samples %ld\n", tid, B, polls,
                tt / leaves * 1e6, worst * 1e3, st.games_completed, st.samples);
    gz_pool_destroy(pool);
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 256;
    const int polls = argc > 2 ? atoi(argv[2]) : 2000;
    const int evals = argc > 3 ? atoi(argv[3]) : 800;
    const int threads = argc > 4 ? atoi(argv[4]) : 1;
    const int spin = argc > 5 ? atoi(argv[5]) : 0;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(run, i, B, polls, evals, spin);
    for (auto& t : ts) t.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%d threads: %.1f s wall, %.0f leaves/s total\n", threads, el, (double)threads * B * polls / el);
    return 0;
}
