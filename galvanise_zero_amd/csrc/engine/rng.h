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
//
// discard(n) advances the generator by n draws whose values nobody reads (the root latch's per-child
// draws in spin playouts, evaluator.cpp:461-475): the count is deferred and applied at the next read
// as one GF(2)-linear jump (xoroshiro128+'s state transition is linear over GF(2); the jump by n is
// the product of the precomputed matrices M^(2^i) for the set bits of n, each applied through
// 4-bit lookup tables), so a spin playout costs no generator steps and the state at every read is
// exactly the state after the same number of single steps.
#pragma once

#include <cstdint>

namespace gz {

// xoroshiro128+ jump tables: kJumpPow powers M^(2^i), each as 32 nibble tables of 16 states
struct RngJumpTables {
    static constexpr int kJumpPow = 44;
    uint64_t t[kJumpPow][32][16][2];
    RngJumpTables();
    static const RngJumpTables& get() {
        static const RngJumpTables tables;
        return tables;
    }
};

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
        pending = 0;
    }

    static uint64_t mix(uint64_t global_seed, uint64_t game_index, uint64_t stream) {
        uint64_t x = global_seed ^ (game_index * 0xD1B54A32D192ED03ull) ^ (stream * 0x8CB92BA72F3D8DD7ull);
        return splitmix64(x);
    }

    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return 0xFFFFFFFFu; }

    // one step of the state transition (also the linear map the jump tables are built from)
    static inline void step(uint64_t& a0, uint64_t& a1) {
        const uint64_t a = a0;
        const uint64_t b = a1 ^ a;
        a0 = rotl(a, 24) ^ b ^ (b << 16);
        a1 = rotl(b, 37);
    }

    void discard(uint64_t n) { pending += n; }

    result_type operator()() {
        if (__builtin_expect(pending != 0, 0)) flush();
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

    bool operator==(const Rng& o) const {
        Rng a = *this, b = o;
        a.flush();
        b.flush();
        return a.s0 == b.s0 && a.s1 == b.s1;
    }

    // apply the deferred discards
    void flush() {
        uint64_t n = pending;
        pending = 0;
        if (n < 64) {
            for (; n > 0; --n) step(s0, s1);
            return;
        }
        const RngJumpTables& J = RngJumpTables::get();
        for (int i = 0; n != 0; ++i, n >>= 1) {
            if (!(n & 1)) continue;
            if (i >= RngJumpTables::kJumpPow) {   // beyond the tables (never in practice): single steps
                for (uint64_t k = n << i; k > 0; --k) step(s0, s1);
                break;
            }
            uint64_t r0 = 0, r1 = 0;
            for (int k = 0; k < 16; ++k) {
                const uint64_t* e = J.t[i][k][(s0 >> (4 * k)) & 15];
                r0 ^= e[0];
                r1 ^= e[1];
            }
            for (int k = 0; k < 16; ++k) {
                const uint64_t* e = J.t[i][16 + k][(s1 >> (4 * k)) & 15];
                r0 ^= e[0];
                r1 ^= e[1];
            }
            s0 = r0;
            s1 = r1;
        }
    }

private:
    static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t s0, s1;
    uint64_t pending = 0;
};

inline RngJumpTables::RngJumpTables() {
    // columns of M^(2^i): the image of each unit state vector (bit j: s0 bit j for j < 64, else s1)
    static uint64_t col[128][2], nxt[128][2];
    for (int j = 0; j < 128; ++j) {
        uint64_t a0 = j < 64 ? 1ull << j : 0, a1 = j < 64 ? 0 : 1ull << (j - 64);
        Rng::step(a0, a1);
        col[j][0] = a0;
        col[j][1] = a1;
    }
    for (int i = 0; i < kJumpPow; ++i) {
        for (int k = 0; k < 32; ++k)
            for (int v = 0; v < 16; ++v) {
                uint64_t r0 = 0, r1 = 0;
                for (int b = 0; b < 4; ++b)
                    if (v >> b & 1) {
                        r0 ^= col[4 * k + b][0];
                        r1 ^= col[4 * k + b][1];
                    }
                t[i][k][v][0] = r0;
                t[i][k][v][1] = r1;
            }
        // M^(2^(i+1)) = M^(2^i) applied to its own columns
        for (int j = 0; j < 128; ++j) {
            uint64_t r0 = 0, r1 = 0;
            for (int b = 0; b < 128; ++b) {
                const uint64_t bit = b < 64 ? (col[j][0] >> b) & 1 : (col[j][1] >> (b - 64)) & 1;
                if (bit) {
                    r0 ^= col[b][0];
                    r1 ^= col[b][1];
                }
            }
            nxt[j][0] = r0;
            nxt[j][1] = r1;
        }
        for (int j = 0; j < 128; ++j) {
            col[j][0] = nxt[j][0];
            col[j][1] = nxt[j][1];
        }
    }
}

}  // namespace gz
