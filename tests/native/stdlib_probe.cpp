// Probe of this image's libstdc++: std::sort permutations on tie-heavy inputs and
// std::gamma_distribution<float> draws driven by the engine's RNG (csrc/engine/rng.h).
// Built and run by tests/test_stdlib_oracle.py to pin oracle/stdlib_ref.py.
#include "../../galvanise_zero_amd/csrc/engine/rng.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
    const char* mode = argv[1];
    if (mode[0] == 's') {   // sort: args n keyrange seed -> prints permutation
        int n = atoi(argv[2]), kr = atoi(argv[3]);
        gz::Rng rng(strtoull(argv[4], 0, 10));
        std::vector<int> key(n), idx(n);
        for (int i = 0; i < n; ++i) { key[i] = rng.getWithMax(kr); idx[i] = i; }
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return key[a] > key[b]; });
        for (int i = 0; i < n; ++i) std::printf("%d %d\n", key[i], idx[i]);
    } else {                // gamma: args alpha count seed -> prints floats (hex)
        float alpha = strtof(argv[2], 0);
        int n = atoi(argv[3]);
        gz::Rng rng(strtoull(argv[4], 0, 10));
        std::gamma_distribution<float> g(alpha, 1.0f);
        for (int i = 0; i < n; ++i) std::printf("%a\n", (double)g(rng));
        std::printf("%u\n", rng());
    }
    return 0;
}
