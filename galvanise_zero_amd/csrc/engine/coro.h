// Stackful coroutines for the leaf-batching scheduler.
//
// Replaces the k273 greenlets (greenlet_t, createGreenlet, greenlet_switch_to; reference
// src/cpp/scheduler.h:6-8,90-101) with a minimal x86-64 context switch (callee-saved registers,
// mxcsr and x87 control word) on mmap'd stacks with a guard page.  Semantics kept from greenlets:
//   * a coroutine runs until it switches to another one;
//   * when its body returns, control passes to its parent (the scheduler's main loop for game
//     coroutines, the poll caller for the main loop);
//   * switching is strictly single-threaded per scheduler (the reference runs every pool's
//     coroutines on the thread that polls it, selfplaymanager.cpp:153-157).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>

namespace gz {

struct Coro {
    void* sp = nullptr;            // saved stack pointer while suspended
    char* stack = nullptr;         // mmap base (incl. guard page), null for a thread's root
    size_t stack_size = 0;
    Coro* parent = nullptr;        // receives control when the body returns
    std::function<void()> body;
    bool dead = false;
    // TSC cycles this coroutine has run (updated when it is switched away from), and the TSC
    // value when it was last switched to: per-game engine time (selfplay.cpp) at one rdtsc a switch
    uint64_t cycles = 0;
    uint64_t resumed_at = 0;
};

// The coroutine currently running on this thread (a per-thread root Coro when none).
Coro* coro_current();

// Create a suspended coroutine that will run `body` the first time it is switched to.
Coro* coro_create(std::function<void()> body, Coro* parent, size_t stack_size = 256 * 1024);

// Switch from the current coroutine to `to`.  Returns when something switches back.
void coro_switch_to(Coro* to);

// TSC cycles the current coroutine has run so far, including its current stretch.
uint64_t coro_cycles_now();

// TSC ticks per second (calibrated once against the steady clock, ~20 ms on first call).
double tsc_hz();

// Free a coroutine (must not be running).  Dead coroutines may be destroyed by anyone.
void coro_destroy(Coro* c);

}  // namespace gz
