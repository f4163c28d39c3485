// Rng::discard(n) (deferred GF(2) jump) must leave the generator exactly where n single steps do.
#include "../../galvanise_zero_amd/csrc/engine/rng.h"

#include <cstdio>

int main() {
    const unsigned long long ns[] = {0, 1, 2, 26, 63, 64, 65, 127, 1000, 5591, 65535, 65536, 123457, 1u << 20, 3000001};
    int bad = 0;
    for (unsigned long long seed = 1; seed <= 3; ++seed)
        for (unsigned long long n : ns) {
            gz::Rng a(gz::Rng::mix(seed, n, 0)), b(gz::Rng::mix(seed, n, 0));
            a.discard(n / 2);
            a.discard(n - n / 2);   // discards accumulate
            gz::Rng c = a;
            for (unsigned long long k = 0; k < n; ++k) b();
            if (!(c == b)) ++bad;   // equality flushes
            for (int k = 0; k < 8; ++k)
                if (a() != b()) { ++bad; break; }
        }
    std::printf("rng jump check: %d mismatches\n", bad);
    return bad != 0;
}
