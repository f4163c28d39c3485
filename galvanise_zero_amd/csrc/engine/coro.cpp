#include "coro.h"

#include <sys/mman.h>
#include <unistd.h>

#include <x86intrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>

// gz_ctx_switch(void** save_sp, void* load_sp): SysV x86-64.  Saves callee-saved GPRs, mxcsr and
// the x87 control word on the current stack, stores rsp into *save_sp, loads load_sp and restores
// the same frame from there.
asm(R"(
    .text
    .globl gz_ctx_switch
    .type gz_ctx_switch, @function
gz_ctx_switch:
    pushq %rbp
    pushq %rbx
    pushq %r12
    pushq %r13
    pushq %r14
    pushq %r15
    subq $8, %rsp
    stmxcsr (%rsp)
    fnstcw 4(%rsp)
    movq %rsp, (%rdi)
    movq %rsi, %rsp
    ldmxcsr (%rsp)
    fldcw 4(%rsp)
    addq $8, %rsp
    popq %r15
    popq %r14
    popq %r13
    popq %r12
    popq %rbx
    popq %rbp
    ret
    .size gz_ctx_switch, .-gz_ctx_switch

    .globl gz_ctx_trampoline
    .type gz_ctx_trampoline, @function
gz_ctx_trampoline:
    movq %r12, %rdi
    call gz_coro_entry
    ud2
    .size gz_ctx_trampoline, .-gz_ctx_trampoline
)");

extern "C" void gz_ctx_switch(void** save_sp, void* load_sp);
extern "C" void gz_ctx_trampoline();

namespace gz {

static thread_local Coro t_root;
// read at every switch: initial-exec (an %fs-relative load, no __tls_get_addr call)
static thread_local Coro* t_current __attribute__((tls_model("initial-exec"))) = nullptr;

Coro* coro_current() {
    if (t_current == nullptr) t_current = &t_root;
    return t_current;
}

extern "C" void gz_coro_entry(Coro* c) {
    c->body();
    c->body = nullptr;
    c->dead = true;
    Coro* p = c->parent;
    while (p != nullptr && p->dead) p = p->parent;
    if (p == nullptr) {
        std::fprintf(stderr, "gz coroutine finished with no live parent\n");
        std::abort();
    }
    t_current = p;
    const uint64_t now = __rdtsc();
    c->cycles += now - c->resumed_at;
    p->resumed_at = now;
    void* dummy;
    gz_ctx_switch(&dummy, p->sp);
    std::abort();   // never resumed
}

Coro* coro_create(std::function<void()> body, Coro* parent, size_t stack_size) {
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    stack_size = (stack_size + page - 1) / page * page;
    const size_t total = stack_size + page;
    void* mem = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (mem == MAP_FAILED) {
        std::perror("gz coro mmap");
        std::abort();
    }
    mprotect(mem, page, PROT_NONE);   // guard page at the low end

    Coro* c = new Coro;
    c->stack = (char*)mem;
    c->stack_size = total;
    c->parent = parent ? parent : coro_current();
    c->body = std::move(body);

    // Initial frame consumed by the restore half of gz_ctx_switch:
    //   [sp+0] mxcsr | x87 cw, [sp+8] r15, r14, r13, r12, rbx, rbp, [sp+56] return address.
    // After `ret` rsp = sp + 64, which must be 16-byte aligned for the trampoline's `call`.
    uintptr_t top = (uintptr_t)mem + total;
    top &= ~(uintptr_t)15;
    uint64_t* sp = (uint64_t*)(top - 64);
    uint32_t* ctl = (uint32_t*)sp;
    ctl[0] = 0x1F80;          // default mxcsr
    ctl[1] = 0x037F;          // default x87 control word
    sp[1] = 0;                // r15
    sp[2] = 0;                // r14
    sp[3] = 0;                // r13
    sp[4] = (uint64_t)c;      // r12 -> trampoline argument
    sp[5] = 0;                // rbx
    sp[6] = 0;                // rbp
    sp[7] = (uint64_t)&gz_ctx_trampoline;
    c->sp = sp;
    return c;
}

void coro_switch_to(Coro* to) {
    Coro* from = coro_current();
    if (from == to) return;
    t_current = to;
    const uint64_t now = __rdtsc();
    from->cycles += now - from->resumed_at;
    to->resumed_at = now;
    gz_ctx_switch(&from->sp, to->sp);
    // resumed: t_current was set by whoever switched to us
}

uint64_t coro_cycles_now() {
    const Coro* c = coro_current();
    return c->cycles + (__rdtsc() - c->resumed_at);
}

double tsc_hz() {
    static const double hz = [] {
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t c0 = __rdtsc();
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        const uint64_t c1 = __rdtsc();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return (double)(c1 - c0) / s;
    }();
    return hz;
}

void coro_destroy(Coro* c) {
    if (!c) return;
    if (c->stack) munmap(c->stack, c->stack_size);
    delete c;
}

}  // namespace gz
