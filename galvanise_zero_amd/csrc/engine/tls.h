// Per-thread singletons reached through an initial-exec TLS pointer: one %fs-relative load per
// access.  (A plain thread_local object in this dlopen'ed library uses the general-dynamic model --
// a __tls_get_addr call per access, 3.4 % of the engine's time in the bench profile,
// profiles/r03l_sprof_report.txt.)  The object is created on a thread's first access and destroyed
// at that thread's exit.
#pragma once

#include <memory>

namespace gz {

template <typename T>
T& tls_instance() {
    static thread_local T* p __attribute__((tls_model("initial-exec"))) = nullptr;
    if (__builtin_expect(p != nullptr, 1)) return *p;
    static thread_local std::unique_ptr<T> owner;
    owner.reset(new T());
    p = owner.get();
    return *p;
}

}  // namespace gz
