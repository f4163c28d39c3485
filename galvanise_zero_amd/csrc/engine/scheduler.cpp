#include "scheduler.h"

#include "transformer.h"

#include <cassert>
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

NetworkScheduler::NetworkScheduler(const GdlBasesTransformer* transformer, int batch_size, float* buf)
    : transformer(transformer), batch_size(batch_size) {
    if (buf) {
        channel_buf = buf;
    } else {
        channel_buf = new float[(size_t)transformer->totalSize() * batch_size];
        owns_buf = true;
    }
}

NetworkScheduler::~NetworkScheduler() {
    for (Coro* c : all_coros) coro_destroy(c);
    if (main_loop) coro_destroy(main_loop);
    if (owns_buf) delete[] channel_buf;
}

// scheduler.cpp:70-124.  (The reference's LRU lookup at :73-85 is never populated; omitted.)
void NetworkScheduler::evaluate(PuctNodeRequest* request) {
    float* buf = channel_buf + channel_buf_indx;
    request->add(buf, transformer);
    channel_buf_indx += transformer->totalSize();

    const int idx = (int)requestors.size();
    requestors.push_back(coro_current());
    request_nodes.push_back(request->target());
    coro_switch_to(main_loop);

    // back: predictions for this batch are in predict_done_event, our row is idx
    GZ_ASSERT(predict_done_event != nullptr && predict_done_event->pred_count > idx);
    ModelResult res;
    for (int ii = 0; ii < transformer->getNumberPolicies(); ii++)
        res.policies[ii] = predict_done_event->policies[ii] + (size_t)idx * transformer->getPolicySize(ii);
    for (int ii = 0; ii < transformer->getNumberRewards(); ii++)
        res.rewards[ii] = predict_done_event->final_scores[(size_t)idx * transformer->getNumberRewards() + ii];
    request->reply(res, transformer);

    // return to the main loop before continuing; it re-queues us as a runnable
    coro_switch_to(main_loop);
}

void NetworkScheduler::yield() {
    yielders.push_back(coro_current());
    coro_switch_to(main_loop);
}

void NetworkScheduler::addRunnable(std::function<void()> f) {
    GZ_ASSERT(main_loop != nullptr);
    Coro* g = coro_create(std::move(f), main_loop);
    all_coros.push_back(g);
    runnables.push_back(g);
}

void NetworkScheduler::createMainLoop() {
    if (main_loop != nullptr) return;   // Player re-arms between moves; a live loop is reused
    main_loop = coro_create([this]() { this->mainLoop(); }, coro_current());
}

static void reap(std::vector<Coro*>& all, Coro* g) {
    for (size_t i = 0; i < all.size(); ++i) {
        if (all[i] == g) {
            all[i] = all.back();
            all.pop_back();
            break;
        }
    }
    coro_destroy(g);
}

void NetworkScheduler::prefetch_reply(int idx) const {
    const PuctNode* node = request_nodes[idx];
    const char* a = reinterpret_cast<const char*>(node);
    const char* b = reinterpret_cast<const char*>(node->cold() + node->num_children);   // hot + cold entries
    for (const char* q = a; q < b; q += 64) __builtin_prefetch(q, 1, 3);
    const int r = node->lead_role_index > 0 ? node->lead_role_index : 0;
    const float* pol = predict_done_event->policies[r] + (size_t)idx * transformer->getPolicySize(r);
    const char* pa = reinterpret_cast<const char*>(pol);
    const char* pb = reinterpret_cast<const char*>(pol + transformer->getPolicySize(r));
    for (const char* q = pa; q < pb; q += 64) __builtin_prefetch(q, 0, 3);
}

// scheduler.cpp:132-205
void NetworkScheduler::mainLoop() {
    while (true) {
        if (cancelled()) break;
        bool jump_to_top = false;
        if (runnables.empty()) {
            if (requestors.empty()) {
                if (!yielders.empty()) {
                    for (Coro* y : yielders) runnables.push_back(y);
                    yielders.clear();
                    continue;
                }
                break;
            }
            jump_to_top = true;
        }
        if (!jump_to_top && requestors.size() == batch_size) jump_to_top = true;

        if (jump_to_top) {
            coro_switch_to(top);
            if (cancelled()) break;
            GZ_ASSERT(predict_done_event->pred_count == (int)requestors.size());
            if (!requestors.empty()) {
                // replies in request order; the next request's node (header and child array, which
                // its reply writes) and its policy row are requested while this one replies: they
                // are cold (hundreds of games per thread) and independent of this reply
                const int n = (int)requestors.size();
                for (int i = 0; i < n; ++i) {
                    if (i + 1 < n) prefetch_reply(i + 1);
                    coro_switch_to(requestors[i]);
                    runnables.push_back(requestors[i]);
                }
                requestors.clear();
                request_nodes.clear();
            }
            if (!yielders.empty()) {
                for (Coro* y : yielders) runnables.push_back(y);
                yielders.clear();
            }
        }

        Coro* g = runnables.front();
        runnables.pop_front();
        coro_switch_to(g);
        if (g->dead) reap(all_coros, g);
    }
}

// scheduler.cpp:207-241
void NetworkScheduler::poll(const PredictDoneEvent* pde, ReadyEvent* ready_event) {
    ready_event->channel_buf = channel_buf;
    if (main_loop == nullptr && cancelled()) {   // cancelled earlier: nothing runs any more
        ready_event->buf_count = 0;
        return;
    }
    GZ_ASSERT(main_loop != nullptr);
    top = coro_current();
    main_loop->parent = top;
    predict_done_event = pde;
    channel_buf_indx = 0;
    coro_switch_to(main_loop);
    predict_done_event = nullptr;

    if (main_loop->dead && cancelled()) channel_buf_indx = 0;   // stopped by cancel(): no batch
    if (channel_buf_indx == 0) {
        GZ_ASSERT(main_loop->dead);
        coro_destroy(main_loop);
        main_loop = nullptr;
    }
    ready_event->buf_count = channel_buf_indx;
}

}  // namespace gz
