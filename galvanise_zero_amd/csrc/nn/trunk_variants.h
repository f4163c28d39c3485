// Registry of the compiled trunk-kernel instantiations (one translation unit per filter count,
// trunk_f64.hip / trunk_f128.hip / trunk_f256.hip, so they compile in parallel).
//
// A trunk kernel is compiled per (F, PT): F = filters rounded up to 64 / 128 / 256 (the host pads
// other filter counts with zero channels), PT = position tiles of 16 (boards of up to 16 * PT
// positions, H and W given at run time).  Variants per geometry: NB boards per workgroup x WPE
// workgroups per CU ("11", "12", "21"), and the split-precision kernel (P = 3, one board per
// workgroup, boards of up to 64 positions).  v2 (pre-activation / squeeze-excite) nets use the
// trunk_kernel_v2 instantiations of the same variants (trunk_f64_v2.hip, trunk_f128_v2.hip; the
// reference's v2 nets have at most 128 filters).
#pragma once

#include "forward_kernel.h"

#include <cstdio>

namespace gznn {

struct KernelChoice {
    const void* fn = nullptr;
    int act_bytes = 0;
    int nb = 1;
    bool single_image = false;
    int resid_bytes = 0;           // global residual scratch per workgroup (0: registers)
    int threads = 256;             // workgroup size (512: trunk_kernel8 / trunk_kernel_w8)
    int groups = 1;                // wave groups (2: trunk_kernel8, a board per group)
    char name[64] = {0};           // the kernel as rocprofv3 names it
};

template <int F, int PTN, int NB, int WPE, int P = 1, bool V2 = false>
KernelChoice kernel_for() {
    KernelChoice k;
    if constexpr (V2) k.fn = (const void*)&trunk_kernel_v2<F, PTN, NB, WPE, P>;
    else k.fn = (const void*)&trunk_kernel<F, PTN, NB, WPE, P>;
    k.act_bytes = Geo<F, PTN, NB, P>::ACT_BYTES;
    k.nb = NB;
    k.single_image = Geo<F, PTN, NB, P>::SI;
    k.resid_bytes = Geo<F, PTN, NB, P>::RESID_BYTES + Geo<F, PTN, NB, P>::LO_BYTES;
    std::snprintf(k.name, sizeof(k.name), "gznn::trunk_kernel%s<%d, %d, %d, %d, %d>", V2 ? "_v2" : "", F, PTN, NB, WPE, P);
    return k;
}

// two wave groups, one board each (variant 22)
template <int F, int PTN, int P>
KernelChoice kernel8_for() {
    KernelChoice k;
    k.fn = (const void*)&trunk_kernel8<F, PTN, P>;
    k.act_bytes = Geo<F, PTN, 1, P, 2>::ACT_BYTES;
    k.nb = 2;
    k.threads = 512;
    k.groups = 2;
    std::snprintf(k.name, sizeof(k.name), "gznn::trunk_kernel8<%d, %d, %d>", F, PTN, P);
    return k;
}

// one group of 8 waves for two boards (variant 24)
template <int F, int PTN, int P>
KernelChoice kernelw8_for() {
    KernelChoice k;
    k.fn = (const void*)&trunk_kernel_w8<F, PTN, P>;
    k.act_bytes = Geo<F, PTN, 2, P, 3>::ACT_BYTES;
    k.nb = 2;
    k.threads = 512;
    std::snprintf(k.name, sizeof(k.name), "gznn::trunk_kernel_w8<%d, %d, %d>", F, PTN, P);
    return k;
}

// two wave groups of two waves, one board each (variant 23)
template <int F, int PTN, int P>
KernelChoice kernelh2_for() {
    KernelChoice k;
    k.fn = (const void*)&trunk_kernel_h2<F, PTN, P>;
    k.act_bytes = Geo<F, PTN, 1, P, 4>::ACT_BYTES;
    k.nb = 2;
    k.groups = 2;
    std::snprintf(k.name, sizeof(k.name), "gznn::trunk_kernel_h2<%d, %d, %d>", F, PTN, P);
    return k;
}

// precision 3: split (hi / lo) operands; otherwise bf16.  v = NB * 10 + WPE; 22 = two boards as two
// groups of four waves (trunk_kernel8).
template <int F, int PTN, bool V2 = false>
KernelChoice variants(int v, int precision) {
    if (precision == 3) {
        // F = 256 split: one board per workgroup in a single image of hi + lo wrapped rows, where
        // that image and the bias table fit the LDS (10 x 10); otherwise (13 x 13: the hi + lo
        // image needs 189 KB) the two-pass kernel (P = 2: one part in the LDS at a time)
        if constexpr (F == 256) {
            if constexpr (Geo<F, PTN, 1, 3>::SI && Geo<F, PTN, 1, 3>::ACT_BYTES + 40 * 1024 <= 160 * 1024 &&
                          !Geo<F, PTN, 1, 3>::RG) {
                if (v == 11) return kernel_for<F, PTN, 1, 1, 3, V2>();
            } else if constexpr (!V2 && Geo<F, PTN, 1, 2>::SI && Geo<F, PTN, 1, 2>::ACT_BYTES + 16 * 1024 <= 160 * 1024) {
                if (v == 11) return kernel_for<F, PTN, 1, 1, 2, V2>();
            }
            return KernelChoice{};
        }
        // F <= 128 on boards of more than 64 positions (up to 19 x 19): one board per workgroup in a
        // single image with one part at a time -- the two-pass kernel (P = 2; at 19 x 19 the hi + lo
        // image would need 201 KB), which also takes v2 nets (the reference's hexLG / hex19 files)
        if constexpr (F <= 128 && PTN > 4) {
            if (v == 11) return kernel_for<F, PTN, 1, 1, 2, V2>();
            return KernelChoice{};
        }
        if constexpr (F <= 128 && PTN <= 4) {
            if constexpr (2 * Geo<F, PTN, 1, 3>::ACT_BYTES + 16 * 1024 <= 160 * 1024) {
                if (v == 11) return kernel_for<F, PTN, 1, 1, 3, V2>();
                // two boards per workgroup (F = 128: 256-byte wrapped rows, hi + lo in 512 bytes)
                if constexpr (Geo<F, PTN, 1, 3>::WRAP && 4 * Geo<F, PTN, 1, 3>::ACT_BYTES + 16 * 1024 <= 160 * 1024) {
                    if (v == 21) return kernel_for<F, PTN, 2, 1, 3, V2>();
                    if constexpr (!V2) {
                        if (v == 22) return kernel8_for<F, PTN, 3>();
                        if constexpr (F == 128) {
                            if (v == 24) return kernelw8_for<F, PTN, 3>();
                            if (v == 23) return kernelh2_for<F, PTN, 3>();
                        }
                    }
                }
            }
        }
        return KernelChoice{};
    }
    if constexpr (4 * Geo<F, PTN, 1>::ACT_BYTES + 16 * 1024 > 160 * 1024) {   // one board per workgroup only
        return v == 11 ? kernel_for<F, PTN, 1, 1, 1, V2>() : KernelChoice{};
    } else {
        switch (v) {
            case 11: return kernel_for<F, PTN, 1, 1, 1, V2>();
            case 12: if constexpr (PTN == 4) return kernel_for<F, PTN, 1, 2, 1, V2>(); else return KernelChoice{};
            case 21:   // (not where the two boards' tiles would spill registers)
                if constexpr (Geo<F, PTN, 2>::LIVE_VGPRS <= 300) return kernel_for<F, PTN, 2, 1, 1, V2>();
                else return KernelChoice{};
            default: return KernelChoice{};
        }
    }
}

KernelChoice trunk_variant_f64(int pt, int v, int precision);
KernelChoice trunk_variant_f128(int pt, int v, int precision);
KernelChoice trunk_variant_f256(int pt, int v, int precision);
KernelChoice trunk_variant_f64_v2(int pt, int v, int precision);
KernelChoice trunk_variant_f128_v2(int pt, int v, int precision);

// padded filter count and position tiles of a board; 0 when not compiled
inline int padded_filters(int F) { return F <= 64 ? 64 : F <= 128 ? 128 : F <= 256 ? 256 : 0; }
constexpr int kMaxPT = 23;   // boards of up to 368 positions (19 x 19)
// Boards beyond 13 x 13 run on the 23-tile kernels (19 x 19; smaller boards leave tiles off the
// board, which read the zero rows and store nothing) with 128 filters (F <= 64 padded up: the
// 64-filter rows are too narrow for the padded layout that fits a 19 x 19 image in the LDS).
constexpr int kLargePT = 23;
inline int kernel_tiles(int pt) { return pt > 11 && pt <= kLargePT ? kLargePT : pt; }
inline int kernel_filters(int F, int pt) {
    const int f = padded_filters(F);
    return pt > 11 && f == 64 ? 128 : f;
}

inline KernelChoice trunk_variant(int fpad, int pt, int v, int precision, bool v2 = false) {
    if (v2) {
        if (fpad == 64) return trunk_variant_f64_v2(pt, v, precision);
        if (fpad == 128) return trunk_variant_f128_v2(pt, v, precision);
        return KernelChoice{};
    }
    if (fpad == 64) return trunk_variant_f64(pt, v, precision);
    if (fpad == 128) return trunk_variant_f128(pt, v, precision);
    if (fpad == 256) return trunk_variant_f256(pt, v, precision);
    return KernelChoice{};
}

}  // namespace gznn
