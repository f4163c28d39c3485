// Native self-play driver for one GPU: the MI355X-native replacement of the reference's
// Python poll loop (cppinterface.py:78-144) + worker threads (supervisor.cpp:79-99, 196-245).
//
// T host threads each own P game pools (SelfPlayManager, via the engine C-ABI).  A pool's planes
// are written by its coroutines straight into pinned host memory; its batch is copied to HBM, run
// through the fused forward and copied back on the pool's own HIP stream, so while the GPU
// evaluates pool k the thread is already doing tree work for pool k+1 (the reference's
// two-managers-per-thread ping-pong, generalised to P).  No Python per batch.
#include "../../../include/gzero_engine.h"
#include "../../../include/gzero_nn.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>


static thread_local std::string g_err;

namespace {

struct Pool {
    gz_pool* pool = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float* h_planes = nullptr;
    float* h_out = nullptr;          // policies then values (pinned)
    float* d_planes = nullptr;
    float* d_out = nullptr;
    std::vector<float*> h_pol, d_pol;
    float* h_val = nullptr;
    float* d_val = nullptr;
    int rows_in_flight = 0;
};

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
    std::atomic<bool> stop{false};
    std::atomic<long> batches{0}, rows{0}, launches{0}, samples_taken{0};
    std::atomic<long> kernel_us{0};
    std::mutex m;
    std::condition_variable cv;
    std::atomic<int> failed{0};
    std::string fail_msg;
};

#define RCHK(x)                                                                            \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            g_err = std::string(#x) + ": " + hipGetErrorString(e_);                        \
            return -1;                                                                     \
        }                                                                                  \
    } while (0)

static int launch_pool(gz_runner* r, Pool& p, int nrows) {
    p.rows_in_flight = nrows;
    if (nrows == 0) return 0;
    RCHK(hipMemcpyAsync(p.d_planes, p.h_planes, (size_t)nrows * r->total_size * 4, hipMemcpyHostToDevice, p.stream));
    RCHK(hipEventRecord(p.ev0, p.stream));
    if (gz_net_forward_device(r->net, p.stream, p.d_planes, nrows, p.d_pol.data(), p.d_val) != 0) {
        g_err = gz_nn_last_error();
        return -1;
    }
    RCHK(hipEventRecord(p.ev1, p.stream));
    for (int i = 0; i < r->num_policies; ++i)
        RCHK(hipMemcpyAsync(p.h_pol[i], p.d_pol[i], (size_t)nrows * r->policy_sizes[i] * 4, hipMemcpyDeviceToHost,
                            p.stream));
    RCHK(hipMemcpyAsync(p.h_val, p.d_val, (size_t)nrows * r->num_values * 4, hipMemcpyDeviceToHost, p.stream));
    return 0;
}

static void thread_main(gz_runner* r, int tid) {
    if (hipSetDevice(r->cfg.device) != hipSuccess) {
        r->failed = 1;
        return;
    }
    const int P = r->cfg.pools_per_thread;
    std::vector<Pool*> mine;
    for (int k = 0; k < P; ++k) mine.push_back(&r->pools[(size_t)tid * P + k]);
    // prime: start the games and produce each pool's first batch
    for (Pool* p : mine) {
        gz_pool_start(p->pool, &r->conf);
        const int rows = gz_pool_poll(p->pool, 0);
        if (launch_pool(r, *p, rows) != 0) {
            std::lock_guard<std::mutex> lk(r->m);
            r->fail_msg = g_err;
            r->failed = 1;
            return;
        }
    }
    while (!r->stop.load(std::memory_order_relaxed)) {
        for (Pool* p : mine) {
            if (hipStreamSynchronize(p->stream) != hipSuccess) {
                std::lock_guard<std::mutex> lk(r->m);
                r->fail_msg = "hipStreamSynchronize failed";
                r->failed = 1;
                return;
            }
            const int done = p->rows_in_flight;
            if (done > 0) {
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, p->ev0, p->ev1) == hipSuccess)
                    r->kernel_us.fetch_add((long)(ms * 1000.0f), std::memory_order_relaxed);
                r->launches.fetch_add(1, std::memory_order_relaxed);
                r->batches.fetch_add(1, std::memory_order_relaxed);
                r->rows.fetch_add(done, std::memory_order_relaxed);
            }
            const int rows = gz_pool_poll(p->pool, done);
            r->samples_taken.fetch_add(gz_pool_take_sample_count(p->pool), std::memory_order_relaxed);
            if (launch_pool(r, *p, rows) != 0) {
                std::lock_guard<std::mutex> lk(r->m);
                r->fail_msg = g_err;
                r->failed = 1;
                return;
            }
        }
        r->cv.notify_all();
    }
    for (Pool* p : mine) (void)hipStreamSynchronize(p->stream);
}

extern "C" const char* gz_runner_last_error(void) { return g_err.c_str(); }

extern "C" gz_runner* gz_runner_create(gz_net* net, const gz_sm* sm, const gz_transformer* t,
                                       const gz_runner_config* cfg, const gz_selfplay_config* conf,
                                       const int* policy_sizes, int num_policies, int num_values) {
    if (!net || !sm || !t || !cfg || !conf || cfg->num_threads < 1 || cfg->pools_per_thread < 1 ||
        cfg->batch_size < 1) {
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
    const int npools = cfg->num_threads * cfg->pools_per_thread;
    r->pools.resize(npools);
    const int B = cfg->batch_size;
    size_t out_per_row = num_values;
    for (int i = 0; i < num_policies; ++i) out_per_row += policy_sizes[i];
    for (int i = 0; i < npools; ++i) {
        Pool& p = r->pools[i];
        bool ok = hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreate(&p.ev0) == hipSuccess && hipEventCreate(&p.ev1) == hipSuccess &&
                  hipHostMalloc((void**)&p.h_planes, (size_t)B * r->total_size * 4, hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc((void**)&p.h_out, (size_t)B * out_per_row * 4, hipHostMallocDefault) == hipSuccess &&
                  hipMalloc((void**)&p.d_planes, (size_t)B * r->total_size * 4) == hipSuccess &&
                  hipMalloc((void**)&p.d_out, (size_t)B * out_per_row * 4) == hipSuccess;
        if (!ok) {
            g_err = "runner allocation failed";
            delete r;   // leaks device buffers on this error path; process is failing anyway
            return nullptr;
        }
        float* ho = p.h_out;
        float* dd = p.d_out;
        for (int k = 0; k < num_policies; ++k) {
            p.h_pol.push_back(ho);
            p.d_pol.push_back(dd);
            ho += (size_t)B * policy_sizes[k];
            dd += (size_t)B * policy_sizes[k];
        }
        p.h_val = ho;
        p.d_val = dd;
        const std::string ident = "gpu" + std::to_string(cfg->device) + "_p" + std::to_string(i);
        p.pool = gz_pool_create(sm, t, B, ident.c_str(), cfg->seed, cfg->game_index_base + (long)i * B, nullptr,
                                p.h_planes, p.h_pol.data(), p.h_val);
        if (!p.pool) {
            g_err = std::string("gz_pool_create: ") + gz_engine_last_error();
            delete r;
            return nullptr;
        }
    }
    return r;
}

extern "C" int gz_runner_start(gz_runner* r) {
    r->stop = false;
    for (int i = 0; i < r->cfg.num_threads; ++i) r->threads.emplace_back(thread_main, r, i);
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

extern "C" int gz_runner_stats_get(gz_runner* r, gz_runner_stats* out) {
    std::memset(out, 0, sizeof(*out));
    out->batches = r->batches.load();
    out->rows = r->rows.load();
    out->kernel_ms = r->kernel_us.load() / 1000.0;
    out->kernel_launches = r->launches.load();
    out->samples = r->samples_taken.load();
    for (Pool& p : r->pools) {
        gz_pool_stats s;
        gz_pool_get_stats(p.pool, &s);   // counters are plain longs written by the owning thread
        out->games_completed += s.games_completed;
        out->games_with_samples += s.games_with_samples;
        out->no_samples += s.no_samples;
        out->resigns += s.resigns;
        out->aborts += s.aborts_game_length;
        out->dupes += s.dupes;
    }
    return r->failed.load() ? -1 : 0;
}

extern "C" int gz_runner_stop(gz_runner* r) {
    r->stop = true;
    for (std::thread& th : r->threads) th.join();
    r->threads.clear();
    return r->failed.load() ? -1 : 0;
}

extern "C" void gz_runner_destroy(gz_runner* r) {
    if (!r) return;
    if (!r->threads.empty()) gz_runner_stop(r);
    (void)hipSetDevice(r->cfg.device);
    for (Pool& p : r->pools) {
        if (p.pool) gz_pool_destroy(p.pool);
        if (p.stream) (void)hipStreamDestroy(p.stream);
        if (p.ev0) (void)hipEventDestroy(p.ev0);
        if (p.ev1) (void)hipEventDestroy(p.ev1);
        if (p.h_planes) (void)hipHostFree(p.h_planes);
        if (p.h_out) (void)hipHostFree(p.h_out);
        if (p.d_planes) (void)hipFree(p.d_planes);
        if (p.d_out) (void)hipFree(p.d_out);
    }
    delete r;
}
