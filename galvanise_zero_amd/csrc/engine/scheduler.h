// Leaf-batching coroutine scheduler.  Restates NetworkScheduler (reference src/cpp/scheduler.h,
// scheduler.cpp:44-241) and the poll events (events.h:7-17):
//   * evaluate(): the calling coroutine writes its input planes at row `requestors.size()` of
//     channel_buf, parks, and is resumed with its row of the predictions;
//   * mainLoop(): runs runnables until batch_size requests are parked or nothing else can run,
//     then returns to the poll caller ("top"); on the next poll resumes the requestors in request
//     order (each consumes its row), queues them, then continues;
//   * poll(): hands predictions in, returns the next batch of planes (buf_count floats, 0 when the
//     main loop has died).
#pragma once

#include "coro.h"
#include "node.h"

#include <atomic>
#include <deque>
#include <functional>
#include <vector>

namespace gz {

class GdlBasesTransformer;

struct PredictDoneEvent {
    int pred_count = 0;
    std::vector<float*> policies;
    float* final_scores = nullptr;
};

struct ReadyEvent {
    int buf_count = 0;
    float* channel_buf = nullptr;
};

class NetworkScheduler {
public:
    // channel_buf may be caller-owned (e.g. pinned host memory feeding the GPU); else allocated.
    NetworkScheduler(const GdlBasesTransformer* transformer, int batch_size, float* channel_buf = nullptr);
    ~NetworkScheduler();

    void evaluate(PuctNodeRequest* request);
    void yield();

    void addRunnable(std::function<void()> f);
    void createMainLoop();
    bool hasMainLoop() const { return main_loop != nullptr; }

    void poll(const PredictDoneEvent* predict_done_event, ReadyEvent* ready_event);

    int batchSize() const { return batch_size; }
    float* channelBuf() { return channel_buf; }

    // Cancellation (the owner's teardown; any thread): the main loop stops at its next turn -- a
    // game coroutine reaches it at its next evaluation or yield, and playoutMain yields every
    // playout once cancelled -- and poll() then returns no rows, at once for every later call.  The
    // suspended games are abandoned (freed with the scheduler); nothing they emitted changes.
    void cancel() { cancelled_.store(true, std::memory_order_relaxed); }
    bool cancelled() const { return cancelled_.load(std::memory_order_relaxed); }

private:
    void mainLoop();
    void prefetch_reply(int idx) const;

    const GdlBasesTransformer* transformer;
    const unsigned int batch_size;

    std::vector<Coro*> requestors;
    std::vector<const PuctNode*> request_nodes;   // the node each requestor waits to have replied
    std::vector<Coro*> yielders;
    std::deque<Coro*> runnables;
    std::vector<Coro*> all_coros;

    Coro* main_loop = nullptr;
    Coro* top = nullptr;

    float* channel_buf = nullptr;
    bool owns_buf = false;
    int channel_buf_indx = 0;

    const PredictDoneEvent* predict_done_event = nullptr;
    std::atomic<bool> cancelled_{false};
};

}  // namespace gz
