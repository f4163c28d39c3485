// Native self-play driver for one GPU: the MI355X-native replacement of the reference's
// Python poll loop (cppinterface.py:78-144) + worker threads (supervisor.cpp:79-99, 196-245).
//
// T engine threads each own P game pools (SelfPlayManager via the engine C-ABI).  A pool's
// coroutines write its planes into the pool's pinned host buffer; the pool is then queued for ONE
// launcher thread, which composes launches from the queue (whole workgroup rounds, splitting a
// pool's batch between two launches when that fills the last round: see Compose), DMAs each
// launch's planes to a per-slot HBM staging buffer on a copy stream, and issues one segmented
// launch of the fused forward (trunk + dense heads in one kernel for the two-image kernels), which
// writes policies / values straight back into the pools' pinned output buffers.  At most two
// launches are in flight on the launch stream, so the next batch accumulates while the GPU runs
// one.  The engine thread meanwhile advances its other pools (the reference's
// two-managers-per-thread ping-pong, P-way).  GZ_RUNNER_ZERO_COPY=1: the kernel reads the pinned
// planes itself (no staging copy; round 1).
#include "../../../include/gzero_engine.h"
#include "../../../include/gzero_nn.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

static thread_local std::string g_err;

namespace {

enum PoolState : int { kEngine = 0, kQueued = 1, kInFlight = 2, kDead = 3 };

struct Pool {
    gz_pool* pool = nullptr;
    float* h_planes = nullptr;       // pinned: written by the engine, read by the kernel
    float* h_out = nullptr;          // pinned: policies then values, written by the kernel
    std::vector<float*> h_pol;
    float* h_val = nullptr;
    int rows = 0;                    // rows of the pool's current batch (set when queued)
    int rows_done = 0;               // rows whose predictions are in h_out (engine side)
    int sub = 0;                     // rows of the current batch already in a launch (launcher only)
    std::chrono::steady_clock::time_point queued_at;   // set under qm when queued
    std::atomic<int> state{kEngine};
    long launched = 0;               // batches whose rows have all been launched (launcher only)
    long queued_batches = 0;         // batches the engine thread has queued (engine only)
    // generation roll with per-pool filters: clear this pool's duplicate filter just before its
    // engine thread delivers batch `clear_at` (its first batch on the new network); -1: none
    std::atomic<long> clear_at{-1};
};

// A launch is a list of parts: rows [row0, row0 + rows) of a pool's batch.  A pool's batch may be
// split over two launches (exact-round composition below); `last` marks the part whose retirement
// completes the pool's batch (launches on one stream retire in order).
struct Part {
    int pool, row0, rows;
    bool last;
};

struct Batch {
    hipEvent_t ev0 = nullptr, evm = nullptr, ev1 = nullptr;
    hipEvent_t evc = nullptr;        // planes copied to d_planes (copy stream)
    hipEvent_t evk = nullptr;        // output staging: the forward's end (ev1 then follows the copies)
    float* d_planes = nullptr;       // device staging of the batch's planes
    size_t d_cap = 0;                // rows d_planes holds
    float* d_out = nullptr;          // output staging: the batch's policies and values in HBM
    size_t d_out_cap = 0;            // rows d_out holds
    std::vector<Part> parts;
    int rows = 0;
};

// Launch composition: kSplit (default) launches whole workgroup rounds, splitting the last pool's
// batch; kSubset (round 2) the subset of whole pools that fills its rounds best; kLegacy (round 1)
// a queue prefix trimmed to whole rounds.  GZ_RUNNER_COMPOSE=split|subset|legacy.
enum Compose : int { kSplit = 0, kSubset = 1, kLegacy = 2 };

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

struct gz_runner {
    gz_runner_config cfg;
    gz_net* net;
    const gz_sm* sm;
    const gz_transformer* t;
    gz_selfplay_config conf;
    int total_size = 0, num_policies = 0, num_values = 0;
    std::vector<int> policy_sizes;
    std::vector<Pool> pools;
    std::vector<std::thread> threads;
    std::thread launcher;
    hipStream_t stream = nullptr;
    // Planes go to HBM by DMA on their own stream (hipMemcpyAsync from the pools' pinned buffers),
    // overlapping the batch in flight, instead of each trunk workgroup gathering its boards over
    // PCIe when it starts (a burst of ~2.6 MB per wave of workgroups with the MFMAs waiting on it).
    // GZ_RUNNER_ZERO_COPY=1: the kernel reads the pinned planes directly (the round-1 path).
    hipStream_t copy_stream = nullptr;
    bool zero_copy = false;
    // Output staging (large policies, e.g. amazons' 3,041 moves): the forward writes its outputs to
    // HBM and a third stream DMAs them to the pools' pinned buffers, overlapping the next launch,
    // instead of the heads kernel writing every row over PCIe itself (4 % of cfg5's GPU time).
    // GZ_RUNNER_OUT_STAGING=0 / 1 overrides the default (on when the policies take >= 1,024 floats
    // per row).
    bool out_staging = false;
    hipStream_t out_stream = nullptr;
    int out_row_floats = 0;
    Compose compose = kSplit;
    Batch batches_ring[2];

    std::mutex qm;                   // guards queue
    std::condition_variable qcv;
    std::deque<int> queue;           // pools waiting for the GPU, in submission order

    std::atomic<bool> stop{false};
    std::atomic<long> batches{0}, rows{0}, launches{0}, samples_taken{0}, segments{0};
    std::atomic<long> kernel_us{0}, trunk_us{0};
    std::atomic<long> engine_idle_us{0};   // summed over engine threads: no pool of the thread ready
    // launches that ran the multi-board trunk variant (rows >= gz_net_large_min_rows)
    std::atomic<long> large_launches{0}, large_rows{0}, large_trunk_us{0}, large_rounds{0};
    std::atomic<long> split_launches{0};   // launches holding part of a pool's batch (kSplit)
    int wave_rows = 0;
    int large_min_rows = 1 << 30;
    std::mutex m;
    std::condition_variable cv;
    std::atomic<int> failed{0};
    std::string fail_msg;
    std::mutex sm_;                  // guards sample_json
    std::string sample_json;         // comma-joined sample objects awaiting gz_runner_fetch_samples
    gz_unique_states* shared_unique = nullptr;   // per_pool_unique_states == 0: one filter for all pools
    std::atomic<int> live_pools{0};  // pools whose main loop is running (not kDead)
    bool started = false;
    // generation roll (gz_runner_update_network): applied by the launcher between launches, when no
    // pool's batch is split, so every batch runs on one network
    std::mutex roll_m;
    std::condition_variable roll_cv;
    // 0 none, 1 pending, 3 claimed by the launcher (applying), 2 applied, -1 failed.  The launcher
    // claims a pending roll (1 -> 3) before reading roll_blob; a timed-out caller withdraws it
    // (1 -> 0) before its blob can be freed, or waits for a claimed one to finish.
    std::atomic<int> roll_state{0};
    const float* roll_blob = nullptr;
    size_t roll_count = 0;
    int roll_device = 0, roll_clear = 0;
    std::string roll_err;
    std::vector<long> roll_batches;  // per pool: batches launched on the previous network
    long roll_launches = 0;          // launches issued on the previous network
    double roll_apply_ms = 0.0;      // the launcher's wall time applying the last roll
};

static void set_failed(gz_runner* r, const std::string& msg) {
    {
        std::lock_guard<std::mutex> lk(r->m);
        if (!r->failed.load()) r->fail_msg = msg;
        r->failed = 1;
    }
    r->stop = true;
    r->qcv.notify_all();
    r->cv.notify_all();
}

// ---- engine threads ---------------------------------------------------------------------------
static void engine_main(gz_runner* r, int tid) {
    const int P = r->cfg.pools_per_thread;
    std::vector<int> mine;
    for (int k = 0; k < P; ++k) mine.push_back(tid * P + k);
    for (int i : mine) gz_pool_start(r->pools[i].pool, &r->conf);
    int idle = 0;
    using clk = std::chrono::steady_clock;
    clk::time_point idle_since{};
    bool idling = false;
    while (!r->stop.load(std::memory_order_relaxed)) {
        bool progressed = false;
        for (int i : mine) {
            Pool& p = r->pools[i];
            if (p.state.load(std::memory_order_acquire) != kEngine) continue;
            {
                // this poll delivers batch queued_batches - 1 (none on the first poll)
                const long ca = p.clear_at.load(std::memory_order_acquire);
                if (ca >= 0 && p.queued_batches > 0 && p.queued_batches - 1 == ca) {
                    if (gz_pool_clear_unique_states(p.pool) != 0) set_failed(r, "clear_unique_states failed");
                    p.clear_at.store(-1, std::memory_order_release);
                }
            }
            const int n = gz_pool_poll(p.pool, p.rows_done);
            if (r->cfg.keep_samples) {
                long cnt = 0;
                char* j = gz_pool_fetch_samples_n(p.pool, &cnt);
                if (j) {
                    const size_t len = std::strlen(j);   // "[{...},{...}]"
                    std::lock_guard<std::mutex> lk(r->sm_);
                    if (len > 2) {
                        if (!r->sample_json.empty()) r->sample_json += ',';
                        r->sample_json.append(j + 1, len - 2);
                    }
                    gz_free(j);
                }
                r->samples_taken.fetch_add(cnt, std::memory_order_relaxed);
            } else {
                r->samples_taken.fetch_add(gz_pool_take_sample_count(p.pool), std::memory_order_relaxed);
            }
            progressed = true;
            if (n <= 0) {                 // main loop ended (never in self-play) or error
                p.state.store(kDead, std::memory_order_release);
                r->live_pools.fetch_sub(1, std::memory_order_relaxed);
                r->qcv.notify_one();
                if (n < 0) set_failed(r, std::string("gz_pool_poll: ") + gz_engine_last_error());
                continue;
            }
            p.rows = n;
            p.queued_batches++;
            p.state.store(kQueued, std::memory_order_release);
            {
                std::lock_guard<std::mutex> lk(r->qm);
                r->pools[i].sub = 0;
                r->pools[i].queued_at = std::chrono::steady_clock::now();
                r->queue.push_back(i);
            }
            r->qcv.notify_one();
        }
        if (progressed) {
            idle = 0;
            if (idling) {
                r->engine_idle_us.fetch_add(
                    std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - idle_since).count(),
                    std::memory_order_relaxed);
                idling = false;
            }
        } else if (!idling) {
            idling = true;
            idle_since = clk::now();
            cpu_relax();
        } else if (++idle < 2000) {
            cpu_relax();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
}

// ---- generation roll ----------------------------------------------------------------------------
// The reference swaps the network between poll loops (worker.py:138-160, Supervisor.update_nn
// cppinterface.py:146-147) and clears the duplicate filter (supervisor_impl.cpp:138-144); here the
// launcher swaps it between two launches.  gz_net_set_weights waits for the launches in flight
// (which finish on the previous image) before freeing it.
static void apply_roll(gz_runner* r, long launches_issued) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = r->roll_device ? gz_net_set_weights_device(r->net, r->roll_blob, r->roll_count)
                                  : gz_net_set_weights(r->net, r->roll_blob, r->roll_count);
    r->roll_apply_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    int rc2 = 0;
    if (rc == 0 && r->roll_clear) {
        if (r->shared_unique) {
            rc2 = gz_unique_states_clear(r->shared_unique);   // one filter for every pool: now
        } else {
            // each pool's own filter: at the pool's first batch on the new network (deterministic)
            for (size_t i = 0; i < r->pools.size(); ++i) r->pools[i].clear_at.store(r->roll_batches[i], std::memory_order_release);
        }
    }
    std::lock_guard<std::mutex> lk(r->roll_m);
    r->roll_launches = launches_issued;
    if (rc != 0 || rc2 != 0) {
        r->roll_err = rc != 0 ? std::string("gz_net_set_weights: ") + gz_nn_last_error() : std::string("clear_unique_states failed");
        r->roll_state = -1;
    } else {
        r->roll_state = 2;
    }
    r->roll_cv.notify_all();
}

// ---- launcher thread --------------------------------------------------------------------------
static void launcher_main(gz_runner* r) {
    if (hipSetDevice(r->cfg.device) != hipSuccess) {
        set_failed(r, "hipSetDevice failed in launcher");
        return;
    }
    const int max_rows = r->cfg.max_launch_rows > 0 ? r->cfg.max_launch_rows : 1 << 30;
    // Launch batching: hold a launch until min_launch_rows rows are queued or its oldest pool has
    // waited max_launch_wait_us - also when the GPU is idle, which in the host-bound regime is most
    // of the time (otherwise single-pool launches dominate).  The engine threads keep working on
    // their other pools meanwhile, and a larger launch runs the two-boards-per-workgroup kernel,
    // which needs half the L2 weight stream per board.
    const int min_rows = r->cfg.min_launch_rows;
    const int wave_rows = gz_net_wave_rows(r->net);   // rows of one full wave of the large kernel
    const auto max_wait = std::chrono::microseconds(r->cfg.max_launch_wait_us > 0 ? r->cfg.max_launch_wait_us : 0);
    std::deque<int> inflight;        // indices into batches_ring, oldest first
    int next_slot = 0;
    long launches_issued = 0;
    std::vector<gz_segment> segs, hsegs;
    while (true) {
        // retire finished batches (in order: one stream)
        while (!inflight.empty()) {
            Batch& b = r->batches_ring[inflight.front()];
            const hipError_t q = hipEventQuery(b.ev1);
            if (q == hipErrorNotReady) break;
            if (q != hipSuccess) {
                set_failed(r, std::string("forward failed: ") + hipGetErrorString(q));
                return;
            }
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, b.ev0, r->out_staging ? b.evk : b.ev1) == hipSuccess)
                r->kernel_us.fetch_add((long)(ms * 1000.0f), std::memory_order_relaxed);
            if (hipEventElapsedTime(&ms, b.ev0, b.evm) == hipSuccess) {
                r->trunk_us.fetch_add((long)(ms * 1000.0f), std::memory_order_relaxed);
                if (b.rows >= r->large_min_rows) {
                    r->large_launches.fetch_add(1, std::memory_order_relaxed);
                    r->large_rows.fetch_add(b.rows, std::memory_order_relaxed);
                    r->large_trunk_us.fetch_add((long)(ms * 1000.0f), std::memory_order_relaxed);
                    if (r->wave_rows > 0)
                        r->large_rounds.fetch_add((b.rows + r->wave_rows - 1) / r->wave_rows, std::memory_order_relaxed);
                }
            }
            for (const Part& pt : b.parts) {
                if (!pt.last) continue;
                Pool& p = r->pools[pt.pool];
                p.rows_done = p.rows;
                p.state.store(kEngine, std::memory_order_release);
            }
            // every counter of a launch is taken when it retires, so a stats snapshot never holds a
            // launch without its rows
            r->launches.fetch_add(1, std::memory_order_relaxed);
            r->segments.fetch_add((long)b.parts.size(), std::memory_order_relaxed);
            if (b.parts.front().row0 > 0 || !b.parts.back().last) r->split_launches.fetch_add(1, std::memory_order_relaxed);
            r->rows.fetch_add(b.rows, std::memory_order_relaxed);
            r->batches.fetch_add(1, std::memory_order_relaxed);
            inflight.pop_front();
            r->cv.notify_all();
        }
        if (r->stop.load(std::memory_order_relaxed)) {
            if (inflight.empty()) return;
            std::this_thread::sleep_for(std::chrono::microseconds(50));
            continue;
        }
        if (inflight.size() >= 2) {
            // both launch slots busy: sleep until the older batch completes (blocking-sync event),
            // leaving the core to the engine threads
            (void)hipEventSynchronize(r->batches_ring[inflight.front()].ev1);
            continue;
        }
        if (r->roll_state.load(std::memory_order_acquire) == 1) {
            bool split_pending;
            {
                std::lock_guard<std::mutex> lk(r->qm);
                split_pending = !r->queue.empty() && r->pools[r->queue.front()].sub > 0;
                if (!split_pending) {
                    r->roll_batches.resize(r->pools.size());
                    for (size_t i = 0; i < r->pools.size(); ++i) r->roll_batches[i] = r->pools[i].launched;
                }
            }
            int pending = 1;
            if (!split_pending && r->roll_state.compare_exchange_strong(pending, 3)) apply_roll(r, launches_issued);
        }
        // gather waiting pools into one segmented launch
        Batch& b = r->batches_ring[next_slot];
        b.parts.clear();
        b.rows = 0;
        {
            std::unique_lock<std::mutex> lk(r->qm);
            if (r->queue.empty()) {
                if (inflight.empty())
                    r->qcv.wait_for(lk, std::chrono::microseconds(200));
                else
                    r->qcv.wait_for(lk, std::chrono::microseconds(30));
            }
            if (r->queue.empty()) continue;
            int queued = 0;                   // rows waiting (a split pool's remainder included)
            for (int i : r->queue) queued += r->pools[i].rows - r->pools[i].sub;
            // no more rows can arrive while no live pool is with its engine thread
            bool all_waiting = true;
            for (const Pool& p : r->pools)
                if (p.state.load(std::memory_order_acquire) == kEngine) {
                    all_waiting = false;
                    break;
                }
            if (min_rows > 0) {
                const auto deadline = r->pools[r->queue.front()].queued_at + max_wait;
                if (queued < min_rows && !all_waiting && (int)r->queue.size() < GZ_MAX_SEGMENTS &&
                    std::chrono::steady_clock::now() < deadline) {
                    // wait for more pools, the deadline, or (next loop) the batch in flight
                    r->qcv.wait_until(lk, std::min(deadline, std::chrono::steady_clock::now() +
                                                                 std::chrono::microseconds(100)));
                    continue;
                }
            }
            if (r->compose == kSplit) {
                // Whole workgroup rounds: the two-boards-per-workgroup trunk runs one workgroup
                // per CU (LDS), so a launch costs ceil(rows / wave_rows) rounds and a partial last
                // round idles CUs (pools hold ~215 rows in the steady state, so whole pools rarely
                // add up to whole rounds).  Launch the largest multiple of wave_rows that is
                // queued, splitting the last pool's batch; its remainder stays at the queue front
                // (re-stamped, so it waits for more rows like a newly queued pool).  Fewer rows
                // than one round, or a queue nothing can join (all_waiting), launch whole.
                int target = std::min(queued, max_rows);
                // a pending generation roll waits for a launch that splits no pool: while one is
                // pending, launches end at a whole-pool boundary (also when max_launch_rows is what
                // limits them), so the queue front soon holds no split pool
                const bool roll_pending = r->roll_state.load() == 1;
                if (wave_rows > 0 && target > wave_rows && !all_waiting && !roll_pending)
                    target = (target / wave_rows) * wave_rows;
                while (!r->queue.empty() && b.rows < target && (int)b.parts.size() < GZ_MAX_SEGMENTS) {
                    const int i = r->queue.front();
                    Pool& p = r->pools[i];
                    const int take = std::min(p.rows - p.sub, target - b.rows);
                    if (roll_pending && take < p.rows - p.sub && !b.parts.empty()) break;
                    const bool last = p.sub + take == p.rows;
                    b.parts.push_back(Part{i, p.sub, take, last});
                    b.rows += take;
                    p.sub += take;
                    if (last) {
                        r->queue.pop_front();
                        p.launched++;
                    } else {
                        p.queued_at = std::chrono::steady_clock::now();
                    }
                }
            } else {
                std::vector<int> pools;
                while (!r->queue.empty() && (int)pools.size() < GZ_MAX_SEGMENTS) {
                    const int i = r->queue.front();
                    if (!pools.empty() && b.rows + r->pools[i].rows > max_rows) break;
                    r->queue.pop_front();
                    pools.push_back(i);
                    b.rows += r->pools[i].rows;
                }
                if (wave_rows > 0 && b.rows > wave_rows) {
                    if (r->compose == kLegacy) {
                        // round 1: trim a queue prefix to exact whole waves
                        const int target = (b.rows / wave_rows) * wave_rows;
                        while (pools.size() > 1 && b.rows > target && b.rows - r->pools[pools.back()].rows >= target) {
                            b.rows -= r->pools[pools.back()].rows;
                            r->queue.push_front(pools.back());
                            pools.pop_back();
                        }
                    } else {
                        // round 2: the subset of the gathered pools -- always with the oldest --
                        // whose rows fill their workgroup rounds best (0/1 subset sums over <= 32
                        // pools), preferring more rounds within 2 % of the best fill; the rest go
                        // back to the queue front in order
                        const int n = (int)pools.size();
                        std::vector<int> rows(n);
                        for (int k = 0; k < n; ++k) rows[k] = r->pools[pools[k]].rows;
                        const int total = b.rows;
                        std::vector<int> from(total + 1, -1);   // item that first reached a sum
                        from[rows[0]] = 0;
                        for (int k = 1; k < n; ++k)
                            for (int sum = total; sum >= rows[k]; --sum)
                                if (from[sum] < 0 && from[sum - rows[k]] >= 0 && sum - rows[k] >= rows[0]) from[sum] = k;
                        const int max_r = (total + wave_rows - 1) / wave_rows;
                        std::vector<int> best_sum(max_r + 1, 0);
                        double best_fill = 0.0;
                        for (int sum = rows[0]; sum <= total; ++sum)
                            if (from[sum] >= 0) best_sum[(sum + wave_rows - 1) / wave_rows] = sum;
                        for (int rr = 1; rr <= max_r; ++rr)
                            if (best_sum[rr] > 0) best_fill = std::max(best_fill, (double)best_sum[rr] / ((double)rr * wave_rows));
                        int pick = 0;
                        for (int rr = max_r; rr >= 1; --rr)
                            if (best_sum[rr] > 0 && (double)best_sum[rr] / ((double)rr * wave_rows) >= best_fill - 0.02) {
                                pick = best_sum[rr];
                                break;
                            }
                        if (pick > 0 && pick < total) {
                            std::vector<char> chosen(n, 0);
                            for (int sum = pick; sum > 0;) {
                                const int k = from[sum];
                                chosen[k] = 1;
                                if (k == 0) break;
                                sum -= rows[k];
                            }
                            std::vector<int> keep, back;
                            for (int k = 0; k < n; ++k) (chosen[k] ? keep : back).push_back(pools[k]);
                            for (auto it = back.rbegin(); it != back.rend(); ++it) r->queue.push_front(*it);
                            pools = keep;
                            b.rows = pick;
                        }
                    }
                }
                for (int i : pools) {
                    r->pools[i].sub = r->pools[i].rows;
                    r->pools[i].launched++;
                    b.parts.push_back(Part{i, 0, r->pools[i].rows, true});
                }
            }
        }
        if (b.parts.empty()) continue;
        if (b.rows == 0) {   // pools with nothing to evaluate: hand them back without a launch
            for (const Part& pt : b.parts) {
                Pool& p = r->pools[pt.pool];
                p.rows_done = p.rows;
                p.state.store(kEngine, std::memory_order_release);
            }
            r->cv.notify_all();
            continue;
        }
        segs.assign(b.parts.size(), gz_segment{});
        for (size_t k = 0; k < b.parts.size(); ++k) {
            const Part& pt = b.parts[k];
            Pool& p = r->pools[pt.pool];
            p.state.store(kInFlight, std::memory_order_relaxed);
            segs[k].rows = pt.rows;
            segs[k].planes = p.h_planes + (size_t)pt.row0 * r->total_size;
            for (int j = 0; j < r->num_policies; ++j) segs[k].policies[j] = p.h_pol[j] + (size_t)pt.row0 * r->policy_sizes[j];
            segs[k].values = p.h_val + (size_t)pt.row0 * r->num_values;
        }
        if (!r->zero_copy) {
            // this slot's previous batch has retired (two slots, retired in order): its staging
            // buffer is free
            const size_t row_floats = (size_t)r->total_size;
            if (b.d_cap < (size_t)b.rows) {
                if (b.d_planes) (void)hipFree(b.d_planes);
                b.d_planes = nullptr;
                const size_t cap = std::max((size_t)b.rows, (size_t)4096);
                if (hipMalloc((void**)&b.d_planes, cap * row_floats * 4) != hipSuccess) {
                    set_failed(r, "device plane staging allocation failed");
                    return;
                }
                b.d_cap = cap;
            }
            size_t off = 0;
            for (gz_segment& sg : segs) {
                if (sg.rows > 0 &&
                    hipMemcpyAsync(b.d_planes + off * row_floats, sg.planes, (size_t)sg.rows * row_floats * 4,
                                   hipMemcpyHostToDevice, r->copy_stream) != hipSuccess) {
                    set_failed(r, "plane copy failed");
                    return;
                }
                sg.planes = b.d_planes + off * row_floats;
                off += sg.rows;
            }
            if (hipEventRecord(b.evc, r->copy_stream) != hipSuccess || hipStreamWaitEvent(r->stream, b.evc, 0) != hipSuccess) {
                set_failed(r, "plane copy event failed");
                return;
            }
        }
        if (r->out_staging) {
            // the segments' outputs to this slot's HBM staging, [segment][policy 0 .. R-1, value]
            // blocks of rows x size; the pinned destinations kept for the copies below
            if (b.d_out_cap < (size_t)b.rows) {
                if (b.d_out) (void)hipFree(b.d_out);
                b.d_out = nullptr;
                const size_t cap = std::max((size_t)b.rows, (size_t)4096);
                if (hipMalloc((void**)&b.d_out, cap * r->out_row_floats * 4) != hipSuccess) {
                    set_failed(r, "device output staging allocation failed");
                    return;
                }
                b.d_out_cap = cap;
            }
            hsegs = segs;
            size_t off = 0;
            for (gz_segment& sg : segs) {
                for (int j = 0; j < r->num_policies; ++j) {
                    sg.policies[j] = b.d_out + off;
                    off += (size_t)sg.rows * r->policy_sizes[j];
                }
                sg.values = b.d_out + off;
                off += (size_t)sg.rows * r->num_values;
            }
        }
        if (hipEventRecord(b.ev0, r->stream) != hipSuccess ||
            gz_net_forward_segments_ev(r->net, r->stream, segs.data(), (int)segs.size(), b.evm) != 0) {
            set_failed(r, std::string("launch failed: ") + gz_nn_last_error());
            return;
        }
        if (r->out_staging) {
            bool ok = hipEventRecord(b.evk, r->stream) == hipSuccess && hipStreamWaitEvent(r->out_stream, b.evk, 0) == hipSuccess;
            for (size_t k = 0; ok && k < segs.size(); ++k) {
                const gz_segment& d = segs[k];
                const gz_segment& h = hsegs[k];
                if (d.rows == 0) continue;
                for (int j = 0; ok && j < r->num_policies; ++j)
                    ok = hipMemcpyAsync(h.policies[j], d.policies[j], (size_t)d.rows * r->policy_sizes[j] * 4,
                                        hipMemcpyDeviceToHost, r->out_stream) == hipSuccess;
                ok = ok && hipMemcpyAsync(h.values, d.values, (size_t)d.rows * r->num_values * 4, hipMemcpyDeviceToHost,
                                          r->out_stream) == hipSuccess;
            }
            if (!ok || hipEventRecord(b.ev1, r->out_stream) != hipSuccess) {
                set_failed(r, "output copy failed");
                return;
            }
        } else if (hipEventRecord(b.ev1, r->stream) != hipSuccess) {
            set_failed(r, "launch event failed");
            return;
        }
        inflight.push_back(next_slot);
        next_slot ^= 1;
        ++launches_issued;
    }
}

extern "C" const char* gz_runner_last_error(void) { return g_err.c_str(); }

extern "C" char* gz_runner_fetch_samples(gz_runner* r) {
    std::string out;
    {
        std::lock_guard<std::mutex> lk(r->sm_);
        if (r->sample_json.empty()) return nullptr;
        out.reserve(r->sample_json.size() + 2);
        out += '[';
        out += r->sample_json;
        out += ']';
        r->sample_json.clear();
    }
    char* c = (char*)std::malloc(out.size() + 1);
    std::memcpy(c, out.c_str(), out.size() + 1);
    return c;
}

extern "C" gz_runner* gz_runner_create(gz_net* net, const gz_sm* sm, const gz_transformer* t,
                                       const gz_runner_config* cfg, const gz_selfplay_config* conf,
                                       const int* policy_sizes, int num_policies, int num_values) {
    if (!net || !sm || !t || !cfg || !conf || cfg->num_threads < 1 || cfg->pools_per_thread < 1 ||
        cfg->batch_size < 1 || num_policies < 1 || num_policies > GZ_MAX_ROLES) {
        g_err = "bad runner arguments";
        return nullptr;
    }
    if (hipSetDevice(cfg->device) != hipSuccess) {
        g_err = "hipSetDevice failed";
        return nullptr;
    }
    gz_runner* r = new gz_runner;
    r->cfg = *cfg;
    r->net = net;
    r->sm = sm;
    r->t = t;
    r->conf = *conf;
    r->total_size = gz_transformer_total_size(t);
    r->num_policies = num_policies;
    r->num_values = num_values;
    r->policy_sizes.assign(policy_sizes, policy_sizes + num_policies);
    r->large_min_rows = gz_net_large_min_rows(net);
    r->wave_rows = gz_net_wave_rows(net);
    bool ok = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&r->copy_stream, hipStreamNonBlocking) == hipSuccess;
    {
        const char* e = std::getenv("GZ_RUNNER_ZERO_COPY");
        r->zero_copy = e != nullptr && e[0] == '1';
        int pol_floats = 0;
        for (int j = 0; j < num_policies; ++j) pol_floats += policy_sizes[j];
        r->out_row_floats = pol_floats + num_values;
        r->out_staging = !r->zero_copy && pol_floats >= 1024;
        if (const char* o = std::getenv("GZ_RUNNER_OUT_STAGING")) r->out_staging = !r->zero_copy && o[0] == '1';
        if (r->out_staging) ok = ok && hipStreamCreateWithFlags(&r->out_stream, hipStreamNonBlocking) == hipSuccess;
        const char* t = std::getenv("GZ_RUNNER_LEGACY_TRIM");
        if (t != nullptr && t[0] == '1') r->compose = kLegacy;
        if (const char* c = std::getenv("GZ_RUNNER_COMPOSE")) {
            const std::string m(c);
            r->compose = m == "subset" ? kSubset : m == "legacy" ? kLegacy : kSplit;
        }
    }
    for (Batch& b : r->batches_ring)
        ok = ok && hipEventCreate(&b.ev0) == hipSuccess && hipEventCreate(&b.evm) == hipSuccess &&
             hipEventCreateWithFlags(&b.ev1, hipEventBlockingSync) == hipSuccess &&
             hipEventCreateWithFlags(&b.evc, hipEventDisableTiming) == hipSuccess && hipEventCreate(&b.evk) == hipSuccess;
    if (!ok) {
        g_err = "stream / event creation failed";
        gz_runner_destroy(r);
        return nullptr;
    }
    const int npools = cfg->num_threads * cfg->pools_per_thread;
    r->pools = std::vector<Pool>(npools);
    const int B = cfg->batch_size;
    {   // every game coroutine maps its own stack + guard page (2 mappings, engine/coro.cpp)
        long max_maps = 65530;
        if (FILE* f = std::fopen("/proc/sys/vm/max_map_count", "r")) {
            if (std::fscanf(f, "%ld", &max_maps) != 1) max_maps = 65530;
            std::fclose(f);
        }
        const long need = 2L * npools * B + 8192;
        if (need > max_maps) {
            g_err = "runner needs about " + std::to_string(need) + " memory mappings for " +
                    std::to_string((long)npools * B) + " game coroutines, vm.max_map_count is " +
                    std::to_string(max_maps) + ": use fewer games per GPU";
            gz_runner_destroy(r);
            return nullptr;
        }
    }
    if (!cfg->per_pool_unique_states) {
        r->shared_unique = gz_unique_states_create(sm, t, 1000);   // supervisor.cpp:31
    }
    size_t out_per_row = num_values;
    for (int i = 0; i < num_policies; ++i) out_per_row += policy_sizes[i];
    for (int i = 0; i < npools; ++i) {
        Pool& p = r->pools[i];
        if (hipHostMalloc((void**)&p.h_planes, (size_t)B * r->total_size * 4, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&p.h_out, (size_t)B * out_per_row * 4, hipHostMallocDefault) != hipSuccess) {
            g_err = "runner pinned allocation failed";
            gz_runner_destroy(r);
            return nullptr;
        }
        float* ho = p.h_out;
        for (int k = 0; k < num_policies; ++k) {
            p.h_pol.push_back(ho);
            ho += (size_t)B * policy_sizes[k];
        }
        p.h_val = ho;
        const std::string ident = "gpu" + std::to_string(cfg->device) + "_p" + std::to_string(i);
        p.pool = gz_pool_create(sm, t, B, ident.c_str(), cfg->seed, cfg->game_index_base + (long)i * B,
                                r->shared_unique, p.h_planes, p.h_pol.data(), p.h_val);
        if (!p.pool) {
            g_err = std::string("gz_pool_create: ") + gz_engine_last_error();
            gz_runner_destroy(r);
            return nullptr;
        }
    }
    return r;
}

extern "C" int gz_runner_start(gz_runner* r) {
    // the pools' games are started by their engine threads; a second start would add a second
    // set of games with the same seeds
    if (r->started) {
        g_err = "runner already started (a stopped runner cannot be restarted: create a new one)";
        return -1;
    }
    r->started = true;
    r->live_pools = (int)r->pools.size();
    r->stop = false;
    r->launcher = std::thread(launcher_main, r);
    for (int i = 0; i < r->cfg.num_threads; ++i) r->threads.emplace_back(engine_main, r, i);
    return 0;
}

// Block until at least `total_batches` forwards have completed (or timeout_s elapses / failure).
extern "C" int gz_runner_wait_batches(gz_runner* r, long total_batches, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(r->m);
    while (r->batches.load() < total_batches) {
        if (r->failed.load()) {
            g_err = r->fail_msg;
            return -1;
        }
        r->cv.wait_for(lk, std::chrono::milliseconds(2));
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s > 0 && el > timeout_s) {
            g_err = "timeout";
            return -2;
        }
    }
    return 0;
}

// Block until at least `total_rows` leaf evaluations have completed.
extern "C" int gz_runner_wait_rows(gz_runner* r, long total_rows, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(r->m);
    while (r->rows.load() < total_rows) {
        if (r->failed.load()) {
            g_err = r->fail_msg;
            return -1;
        }
        r->cv.wait_for(lk, std::chrono::milliseconds(2));
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s > 0 && el > timeout_s) {
            g_err = "timeout";
            return -2;
        }
    }
    return 0;
}

extern "C" int gz_runner_stats_get(gz_runner* r, gz_runner_stats* out) {
    std::memset(out, 0, sizeof(*out));
    out->batches = r->batches.load();
    out->rows = r->rows.load();
    out->kernel_ms = r->kernel_us.load() / 1000.0;
    out->trunk_ms = r->trunk_us.load() / 1000.0;
    out->engine_idle_ms = r->engine_idle_us.load() / 1000.0;
    out->large_launches = r->large_launches.load();
    out->large_rows = r->large_rows.load();
    out->large_trunk_ms = r->large_trunk_us.load() / 1000.0;
    out->large_rounds = r->large_rounds.load();
    out->split_launches = r->split_launches.load();
    out->kernel_launches = r->launches.load();
    out->samples = r->samples_taken.load();
    out->segments = r->segments.load();
    for (Pool& p : r->pools) {
        if (!p.pool) continue;
        gz_pool_stats s;
        gz_pool_get_stats(p.pool, &s);   // counters are plain longs written by the owning thread
        out->games_completed += s.games_completed;
        out->games_with_samples += s.games_with_samples;
        out->no_samples += s.no_samples;
        out->resigns += s.resigns;
        out->aborts += s.aborts_game_length;
        out->dupes += s.dupes;
        out->completed_game_evals += s.completed_game_evals;
        out->tree_playouts += s.tree_playouts;
    }
    return r->failed.load() ? -1 : 0;
}

extern "C" int gz_runner_stop(gz_runner* r) {
    r->stop = true;
    r->qcv.notify_all();
    // an engine thread inside gz_pool_poll returns at its pool's next coroutine switch: a game that
    // spins without evaluations (playoutMain, evaluator.cpp:744-886) would otherwise hold it until
    // the spin ends -- minutes on few-slot or deep-config runners.  The games in progress are
    // abandoned (a stopped runner cannot be restarted); samples already emitted are unchanged.
    for (Pool& p : r->pools)
        if (p.pool) gz_pool_cancel(p.pool);
    for (std::thread& th : r->threads) th.join();
    r->threads.clear();
    if (r->launcher.joinable()) r->launcher.join();   // drains the batches in flight
    if (r->failed.load()) {
        g_err = r->fail_msg;
        return -1;
    }
    return 0;
}

extern "C" void gz_runner_destroy(gz_runner* r) {
    if (!r) return;
    if (!r->threads.empty() || r->launcher.joinable()) gz_runner_stop(r);
    (void)hipSetDevice(r->cfg.device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    for (Pool& p : r->pools) {
        if (p.pool) gz_pool_destroy(p.pool);
        if (p.h_planes) (void)hipHostFree(p.h_planes);
        if (p.h_out) (void)hipHostFree(p.h_out);
    }
    if (r->copy_stream) (void)hipStreamSynchronize(r->copy_stream);
    if (r->out_stream) (void)hipStreamSynchronize(r->out_stream);
    for (Batch& b : r->batches_ring) {
        if (b.ev0) (void)hipEventDestroy(b.ev0);
        if (b.ev1) (void)hipEventDestroy(b.ev1);
        if (b.evm) (void)hipEventDestroy(b.evm);
        if (b.evc) (void)hipEventDestroy(b.evc);
        if (b.evk) (void)hipEventDestroy(b.evk);
        if (b.d_planes) (void)hipFree(b.d_planes);
        if (b.d_out) (void)hipFree(b.d_out);
    }
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->copy_stream) (void)hipStreamDestroy(r->copy_stream);
    if (r->out_stream) (void)hipStreamDestroy(r->out_stream);
    gz_unique_states_destroy(r->shared_unique);
    delete r;
}

// clear_unique_states at a generation roll (supervisor_impl.cpp:138-144, worker.py:160): the
// shared filter, or every pool's own one (UniqueStates locks, so the engine threads may be running)
extern "C" int gz_runner_clear_unique_states(gz_runner* r) {
    if (!r) return -1;
    if (r->shared_unique) return gz_unique_states_clear(r->shared_unique);
    for (Pool& p : r->pools)
        if (p.pool && gz_pool_clear_unique_states(p.pool) != 0) {
            g_err = gz_engine_last_error();
            return -1;
        }
    return 0;
}

// Generation roll on a live runner: the launcher applies the new weights between two launches
// (no pool batch runs on two networks) and, if asked, clears the duplicate filters; blocks until
// applied.  Before start / after stop the weights are set directly.
extern "C" int gz_runner_update_network(gz_runner* r, const float* blob, size_t count, int device_blob,
                                        int clear_unique_states, double timeout_s) {
    if (!r || !blob) {
        g_err = "null argument";
        return -1;
    }
    const bool live = r->started && r->launcher.joinable() && !r->stop.load();
    if (!live) {
        const int rc = device_blob ? gz_net_set_weights_device(r->net, blob, count) : gz_net_set_weights(r->net, blob, count);
        if (rc != 0) {
            g_err = gz_nn_last_error();
            return -1;
        }
        r->roll_batches.assign(r->pools.size(), 0);
        for (size_t i = 0; i < r->pools.size(); ++i) r->roll_batches[i] = r->pools[i].launched;
        r->roll_launches = r->launches.load();
        if (clear_unique_states && gz_runner_clear_unique_states(r) != 0) return -1;
        return 0;
    }
    std::unique_lock<std::mutex> lk(r->roll_m);
    // one caller at a time: any state but 0 means another caller owns the roll (pending, being
    // applied, or applied / failed and not yet collected -- that caller resets it to 0 on return)
    if (r->roll_state.load() != 0) {
        g_err = "a generation roll is already pending";
        return -1;
    }
    r->roll_blob = blob;
    r->roll_count = count;
    r->roll_device = device_blob;
    r->roll_clear = clear_unique_states;
    r->roll_state = 1;
    r->qcv.notify_all();
    const auto t0 = std::chrono::steady_clock::now();
    while (r->roll_state.load() == 1 || r->roll_state.load() == 3) {
        r->roll_cv.wait_for(lk, std::chrono::milliseconds(2));
        const bool timed_out =
            timeout_s > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s;
        if (r->failed.load() || timed_out) {
            // withdraw the roll before returning (the caller may free the blob); one the launcher
            // has already claimed is waited for -- apply_roll takes no unbounded wait
            int pending = 1;
            if (r->roll_state.compare_exchange_strong(pending, 0)) {
                r->roll_blob = nullptr;
                g_err = r->failed.load() ? r->fail_msg : "timeout waiting for the launcher to apply the generation roll";
                return r->failed.load() ? -1 : -2;
            }
            if (r->roll_state.load() == 3) continue;   // being applied: finishes shortly
        }
    }
    r->roll_blob = nullptr;
    if (r->roll_state.load() < 0) {
        g_err = r->roll_err;
        r->roll_state = 0;
        return -1;
    }
    r->roll_state = 0;
    return 0;
}

// Per-ordinal game costs summed over the runner's pools (gzero_engine.h gz_ordinal_stats).
extern "C" int gz_runner_ordinal_stats(gz_runner* r, gz_ordinal_stats* out) {
    if (!r || !out) {
        g_err = "null argument";
        return -1;
    }
    std::memset(out, 0, sizeof(*out));
    for (Pool& p : r->pools)
        if (p.pool && gz_pool_add_ordinal_stats(p.pool, out) != 0) {
            g_err = gz_engine_last_error();
            return -1;
        }
    return 0;
}

extern "C" double gz_runner_roll_apply_ms(gz_runner* r) { return r ? r->roll_apply_ms : -1.0; }

// After gz_runner_update_network: per pool, the batches launched on the previous network (the
// pool's batches 0 .. pool_batches[i]-1 ran on it, the later ones on the new one), and the launches
// issued before the swap.
extern "C" int gz_runner_roll_info(gz_runner* r, long* pool_batches, int npools, long* launches_before) {
    if (!r) return -1;
    for (int i = 0; i < npools && i < (int)r->roll_batches.size(); ++i) pool_batches[i] = r->roll_batches[i];
    if (launches_before) *launches_before = r->roll_launches;
    return 0;
}
