// Seeded xoroshiro128+ generator with the interface the reference uses from
// K273::xoroshiro128plus32 (k273, not vendored; used at evaluator.h:159, selfplay.h:90):
//   operator()() -> uint32  (also a UniformRandomBitGenerator for std::gamma_distribution,
//                            evaluator.cpp:1249)
//   get()        -> double in [0, 1)
//   getWithMax(n)-> uint32 in [0, n)
// The reference default-constructs (never seeds) these; here every generator is seeded from
// (global seed, game index, stream id) so self-play is reproducible and independent of how games
// are assigned to pools, threads or GPUs.  Exact k273 bit streams are not reproducible (k273 is
// absent): RNG-dependent behaviour is "parity unpinned" against the reference, pinned against
// oracle/puct_ref.py which restates this generator.
#pragma once

#include <cstdint>

namespace gz {

inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

class Rng {
public:
    typedef uint32_t result_type;

    explicit Rng(uint64_t seed = 0x853c49e6748fea9bull) { this->seed(seed); }

    void seed(uint64_t seed) {
        uint64_t x = seed;
        s0 = splitmix64(x);
        s1 = splitmix64(x);
        if (s0 == 0 && s1 == 0) s1 = 1;
    }

    static uint64_t mix(uint64_t global_seed, uint64_t game_index, uint64_t stream) {
        uint64_t x = global_seed ^ (game_index * 0xD1B54A32D192ED03ull) ^ (stream * 0x8CB92BA72F3D8DD7ull);
        return splitmix64(x);
    }

    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return 0xFFFFFFFFu; }

    result_type operator()() {
        const uint64_t a = s0;
        uint64_t b = s1;
        const uint64_t result = a + b;
        b ^= a;
        s0 = rotl(a, 24) ^ b ^ (b << 16);
        s1 = rotl(b, 37);
        return (result_type)(result >> 32);
    }

    double get() { return (double)(*this)() * (1.0 / 4294967296.0); }

    uint32_t getWithMax(uint32_t upper) { return upper ? (*this)() % upper : 0; }

    bool operator==(const Rng& o) const { return s0 == o.s0 && s1 == o.s1; }

private:
    static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t s0, s1;
};

}  // namespace gz
