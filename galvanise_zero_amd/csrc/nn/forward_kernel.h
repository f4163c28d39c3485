// Fused whole-network forward of the v1 residual policy/value CNN for gfx950 (MI355X).
//
// One workgroup (4 waves) evaluates NB boards end to end:
//   planes (fp32 NCHW, HBM) -> im2col in LDS -> initial conv -> B residual blocks -> heads
//   -> softmax policies / value (fp32, HBM).
// Trunk activations never leave the CU: the bf16 copy that feeds the next conv lives in LDS
// (two ping-pong images), the fp32 residual stream lives in the MFMA accumulator registers.
// Weights (bf16, BN folded, MFMA-fragment packed) stream from L2 straight into VGPRs.
//
// Each 3x3 conv is an implicit GEMM  out[co][p] = sum_{tap,ci} W[co][tap,ci] * X[nbr(p,tap)][ci]
// on v_mfma_f32_16x16x32_bf16 with A = weights (rows co), B = activations (cols = positions), so
// the accumulator of a lane holds 4 consecutive channels of one position and the epilogue is one
// 8-byte LDS store.  Wave w owns output channels [w*F/4, (w+1)*F/4) for every position of the
// workgroup's NB boards, so one weight fragment (16 B/lane from L2) feeds NB*ceil(HW/16) MFMAs.
//
// Reference semantics: src/ggpzero/nn/model.py:25-75, 154-296 (see oracle/nn_ref.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gznn {

constexpr int kMaxRoles = 4;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct KParams {
    const __bf16* w0;        // initial conv, packed [K0/32][F][32]
    const float* b0;         // [F]
    const __bf16* wres;      // trunk convs, packed [2B][9][F/32][F][32]
    const float* bres;       // [2B][F]
    const float* wh;         // head 1x1 convs (BN folded) [2R+1][F]
    const float* bh;         // [2R+1]
    const float* pd[kMaxRoles];   // policy dense [2HW][P_r]
    const float* pb[kMaxRoles];   // [P_r]
    const float* vhw;        // value hidden [HW][VH]
    const float* vhb;        // [VH]
    const float* vdw;        // value dense [VH][V]
    const float* vdb;        // [V]
    float* pol[kMaxRoles];   // outputs [n][P_r]
    float* val;              // outputs [n][V]
    int n;                   // boards in this launch
    int C, K0, B, R, VH, V, leaky, flatten_nchw, maxP;
    int P[kMaxRoles];
};

__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }

template <int F, int H, int W, int NB = 1>
struct Geo {
    static constexpr int NPOS = H * W;
    static constexpr int PT = (NPOS + 15) / 16;      // position tiles per board (MFMA N)
    static constexpr int TT = NB * PT;               // position tiles per wave (all boards)
    static constexpr int CT = F / 64;                // co tiles per wave (MFMA M)
    static constexpr int KC = F / 32;                // k-steps per tap
    static constexpr int ROWB = F * 2;               // bytes per LDS activation row
    static constexpr int CPR = F / 8;                // 16-byte chunks per row
    static constexpr int SWZ = (CPR < 16 ? CPR : 16) - 1;
    static constexpr int ACT_BYTES = align16((NPOS + 1) * ROWB);   // + one all-zero row
    static_assert(F % 64 == 0, "filters must be a multiple of 64");
};

// Scratch bytes needed beyond the two activation images (host and device agree on this).
__host__ __device__ inline int scratch_bytes(int npos, int C, int K0, int R, int maxP, int VH) {
    int in_stage = align16(C * npos * 4) + align16((npos + 1) * K0 * 2);
    int hc = 2 * R + 1;
    int heads = align16(4 * hc * npos * 4) + align16(hc * npos * 4)
              + align16((maxP > VH ? maxP : VH) * 4) + 64 * 4;
    return in_stage > heads ? in_stage : heads;
}

__device__ __forceinline__ float act_fn(float v, int leaky) {
    return v > 0.f ? v : (leaky ? 0.03f * v : 0.f);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    __bf16 x = (__bf16)a, y = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

template <int F, int H, int W>
__device__ __forceinline__ void store_act(char* X, int p, int co, f32x4 v) {
    using G = Geo<F, H, W>;
    if (p < G::NPOS) {
        uint2 u;
        u.x = pack2(v[0], v[1]);
        u.y = pack2(v[2], v[3]);
        *(uint2*)(X + p * G::ROWB + ((((co >> 3) ^ (p & G::SWZ))) << 4) + (co & 7) * 2) = u;
    }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Workgroup reduction through an LDS slot per wave; all threads get the result.
template <bool IS_MAX, int NWAVES>
__device__ __forceinline__ float block_reduce(float v, float* red) {
    v = IS_MAX ? wave_max(v) : wave_sum(v);
    const int wave = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wave] = v;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int w = 1; w < NWAVES; ++w) r = IS_MAX ? fmaxf(r, red[w]) : r + red[w];
    return r;
}

// One 3x3 'same' conv over the NB LDS images at X (board b at X + b*ACT_BYTES):
// acc[ct][t] = W * X (fp32 accumulate), tile t = b*PT + pt.  Every weight fragment loaded from L2
// feeds TT = NB*PT MFMAs -- NB is the weight-reuse factor that sets the L2->CU byte rate.
template <int F, int H, int W, int NB>
__device__ __forceinline__ void conv3x3(const char* __restrict__ X, const __bf16* __restrict__ wp,
                                        f32x4 (&acc)[Geo<F, H, W>::CT][Geo<F, H, W, NB>::TT],
                                        int co_base, int li, int g) {
    using G = Geo<F, H, W, NB>;
    constexpr int CT = G::CT, PT = G::PT, TT = G::TT, KC = G::KC;
    // weight prefetch depth in k-steps; D | KC keeps the ring index a compile-time constant while
    // the tap loop stays rolled (a rolled tap loop keeps the LDS address math out of registers)
    constexpr int D = KC < 4 ? KC : 4;
    static_assert(KC % D == 0, "prefetch depth must divide the k-steps per tap");
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // lane's fragment of step s = tap*KC + kc: wp + ((s*F + co_base + 16ct + li) * 32 + 8g)
    const __bf16* wl = wp + (size_t)(co_base + li) * 32 + 8 * g;
    bf16x8 ring[D][CT];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
            ring[d][ct] = *(const bf16x8*)(wl + ((size_t)d * F + 16 * ct) * 32);

#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        int qoff[PT], qswz[PT];
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
            const int p = 16 * pt + li;
            const int y = p / W + dy, x = p % W + dx;
            const bool ok = p < G::NPOS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            const int q = ok ? p + dy * W + dx : G::NPOS;
            qoff[pt] = q * G::ROWB;
            qswz[pt] = q & G::SWZ;
        }
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            bf16x8 b[TT];
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int off = qoff[pt] + (((kc * 4 + g) ^ qswz[pt]) << 4);
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) b[bb * PT + pt] = *(const bf16x8*)(X + bb * G::ACT_BYTES + off);
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int t = 0; t < TT; ++t)
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[kc % D][ct], b[t], acc[ct][t], 0, 0, 0);
            // prefetch step s + D (clamped to the last step: the tail re-reads it harmlessly)
            int sn = tap * KC + kc + D;
            sn = sn < 9 * KC ? sn : 9 * KC - 1;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                ring[kc % D][ct] = *(const bf16x8*)(wl + ((size_t)sn * F + 16 * ct) * 32);
        }
    }
}

// NB boards per workgroup of 4 waves; WPE = minimum resident waves per SIMD the register
// allocation must allow (amdgpu_waves_per_eu), i.e. WPE workgroups per CU.
template <int F, int H, int W, int NB, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
forward_kernel(KParams kp, const float* __restrict__ planes) {
    using G = Geo<F, H, W, NB>;
    constexpr int NPOS = G::NPOS, PT = G::PT, TT = G::TT, CT = G::CT, kThreads = 256;
    constexpr int ACT = G::ACT_BYTES;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* X0 = smem;                 // [NB][ACT]
    char* X1 = smem + NB * ACT;      // [NB][ACT]
    char* SCR = X1;                  // scratch aliases X1 while X1 holds no live activations

    const int board0 = blockIdx.x * NB;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int co_base = wave * (F / 4);
    const int C = kp.C, K0 = kp.K0;

    f32x4 acc[CT][TT];
    f32x4 resid[CT][TT];

    for (int i = tid; i < NB * G::ROWB / 4; i += kThreads) {
        const int bb = i / (G::ROWB / 4), j = i % (G::ROWB / 4);
        ((uint32_t*)(X0 + bb * ACT + NPOS * G::ROWB))[j] = 0u;
    }

    // ---- per board: stage planes, im2col, initial conv (GEMM over K0) ----------------------
    float* sin = (float*)SCR;
    char* IM = SCR + align16(C * NPOS * 4);
    const int imrow = K0 * 2;
    const int imswz = ((K0 >> 3) < 16 ? (K0 >> 3) : 16) - 1;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const bool live = board0 + bb < kp.n;
        const float* in = planes + (size_t)(board0 + bb) * C * NPOS;
        for (int i = tid; i < C * NPOS; i += kThreads) sin[i] = live ? in[i] : 0.f;
        __syncthreads();
        // IM[p][k], k = tap*C + c, zero padded to K0
        for (int i = tid; i < (NPOS + 1) * K0; i += kThreads) {
            const int p = i / K0, k = i - (i / K0) * K0;
            float v = 0.f;
            if (p < NPOS && k < 9 * C) {
                const int tap = k / C, c = k - (k / C) * C;
                const int y = p / W + tap / 3 - 1, x = p % W + tap % 3 - 1;
                if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) v = sin[c * NPOS + y * W + x];
            }
            *(__bf16*)(IM + p * imrow + ((((k >> 3) ^ (p & imswz))) << 4) + (k & 7) * 2) = (__bf16)v;
        }
        __syncthreads();

#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) acc[ct][bb * PT + pt] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < (K0 >> 5); ++s) {
            bf16x8 a[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                a[ct] = *(const bf16x8*)(kp.w0 + ((size_t)(s * F + co_base + 16 * ct + li)) * 32 + 8 * g);
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int p = 16 * pt + li;
                const int q = p < NPOS ? p : NPOS;
                const bf16x8 b = *(const bf16x8*)(IM + q * imrow + ((((s * 4 + g)) ^ (q & imswz)) << 4));
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
                    acc[ct][bb * PT + pt] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct], b, acc[ct][bb * PT + pt], 0, 0, 0);
            }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(kp.b0 + co);
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                f32x4 v = acc[ct][bb * PT + pt];
                v[0] = act_fn(v[0] + bias.x, kp.leaky);
                v[1] = act_fn(v[1] + bias.y, kp.leaky);
                v[2] = act_fn(v[2] + bias.z, kp.leaky);
                v[3] = act_fn(v[3] + bias.w, kp.leaky);
                resid[ct][bb * PT + pt] = v;
                store_act<F, H, W>(X0 + bb * ACT, 16 * pt + li, co, v);
            }
        }
        __syncthreads();    // scratch is reused by the next board
    }
    for (int i = tid; i < NB * G::ROWB / 4; i += kThreads) {
        const int bb = i / (G::ROWB / 4), j = i % (G::ROWB / 4);
        ((uint32_t*)(X1 + bb * ACT + NPOS * G::ROWB))[j] = 0u;
    }
    __syncthreads();

    // ---- residual tower ------------------------------------------------------------------
    constexpr size_t conv_elems = (size_t)9 * F * F;
    for (int blk = 0; blk < kp.B; ++blk) {
        const __bf16* w_a = kp.wres + (size_t)(2 * blk) * conv_elems;
        const __bf16* w_b = w_a + conv_elems;
        const float* b_a = kp.bres + (size_t)(2 * blk) * F;
        const float* b_b = b_a + F;

        conv3x3<F, H, W, NB>(X0, w_a, acc, co_base, li, g);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(b_a + co);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 v = acc[ct][t];
                v[0] = act_fn(v[0] + bias.x, kp.leaky);
                v[1] = act_fn(v[1] + bias.y, kp.leaky);
                v[2] = act_fn(v[2] + bias.z, kp.leaky);
                v[3] = act_fn(v[3] + bias.w, kp.leaky);
                store_act<F, H, W>(X1 + (t / PT) * ACT, 16 * (t % PT) + li, co, v);
            }
        }
        __syncthreads();

        conv3x3<F, H, W, NB>(X1, w_b, acc, co_base, li, g);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(b_b + co);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 v = acc[ct][t];
                const f32x4 r = resid[ct][t];
                v[0] = act_fn(v[0] + bias.x + r[0], kp.leaky);
                v[1] = act_fn(v[1] + bias.y + r[1], kp.leaky);
                v[2] = act_fn(v[2] + bias.z + r[2], kp.leaky);
                v[3] = act_fn(v[3] + bias.w + r[3], kp.leaky);
                resid[ct][t] = v;
                store_act<F, H, W>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co, v);
            }
        }
        __syncthreads();
    }

    // ---- heads, one board at a time: 1x1 convs (2 per policy role + 1 value) from the fp32
    // residual registers, then the dense layers + softmaxes in fp32 -------------------------
    const int HC = 2 * kp.R + 1;
    float* hpart = (float*)SCR;                                  // [4][HC][NPOS]
    float* feat = (float*)(SCR + align16(4 * HC * NPOS * 4));    // [HC][NPOS] flattened per head
    float* lg = (float*)((char*)feat + align16(HC * NPOS * 4));  // logits / hidden scratch
    float* red = (float*)((char*)lg + align16((kp.maxP > kp.VH ? kp.maxP : kp.VH) * 4));
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const int board = board0 + bb;
        const bool live = board < kp.n;
        for (int h = 0; h < HC; ++h) {
            float wv[CT][4];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const float4 w4 = *(const float4*)(kp.wh + (size_t)h * F + co_base + 16 * ct + 4 * g);
                wv[ct][0] = w4.x; wv[ct][1] = w4.y; wv[ct][2] = w4.z; wv[ct][3] = w4.w;
            }
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                float s = 0.f;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s += resid[ct][bb * PT + pt][r] * wv[ct][r];
                s += __shfl_xor(s, 16, 64);
                s += __shfl_xor(s, 32, 64);
                const int p = 16 * pt + li;
                if (g == 0 && p < NPOS) hpart[(wave * HC + h) * NPOS + p] = s;
            }
        }
        __syncthreads();
        for (int i = tid; i < HC * NPOS; i += kThreads) {
            const int h = i / NPOS, p = i - (i / NPOS) * NPOS;
            float s = kp.bh[h];
#pragma unroll
            for (int w = 0; w < 4; ++w) s += hpart[(w * HC + h) * NPOS + p];
            s = act_fn(s, kp.leaky);
            if (h < 2 * kp.R) {
                const int r = h >> 1, c = h & 1;
                const int idx = kp.flatten_nchw ? c * NPOS + p : p * 2 + c;
                feat[r * 2 * NPOS + idx] = s;
            } else {
                feat[2 * kp.R * NPOS + p] = s;
            }
        }
        __syncthreads();

        // policy heads: Dense(2HW -> P_r) + softmax
        for (int r = 0; r < kp.R; ++r) {
            const int P = kp.P[r];
            const float* pf = feat + r * 2 * NPOS;
            const float* wd = kp.pd[r];
            float lmax = -3.0e38f;
            for (int j = tid; j < P; j += kThreads) {
                float z = kp.pb[r][j];
                for (int i = 0; i < 2 * NPOS; ++i) z += pf[i] * wd[(size_t)i * P + j];
                lg[j] = z;
                lmax = fmaxf(lmax, z);
            }
            const float m = block_reduce<true, 4>(lmax, red);
            float lsum = 0.f;
            for (int j = tid; j < P; j += kThreads) {
                const float e = __expf(lg[j] - m);
                lg[j] = e;
                lsum += e;
            }
            const float ssum = block_reduce<false, 4>(lsum, red);
            const float inv = 1.f / ssum;
            if (live) {
                float* out = kp.pol[r] + (size_t)board * P;
                for (int j = tid; j < P; j += kThreads) out[j] = lg[j] * inv;
            }
            __syncthreads();
        }

        // value head: Dense(HW -> VH) + act, Dense(VH -> V) + softmax
        const float* vf = feat + 2 * kp.R * NPOS;
        for (int k = tid; k < kp.VH; k += kThreads) {
            float z = kp.vhb[k];
            for (int p = 0; p < NPOS; ++p) z += vf[p] * kp.vhw[(size_t)p * kp.VH + k];
            lg[k] = act_fn(z, kp.leaky);
        }
        __syncthreads();
        if (wave < kp.V) {
            float s = 0.f;
            for (int k = lane; k < kp.VH; k += 64) s += lg[k] * kp.vdw[(size_t)k * kp.V + wave];
            s = wave_sum(s);
            if (lane == 0) red[16 + wave] = s + kp.vdb[wave];
        }
        __syncthreads();
        if (tid == 0 && live) {
            float m = red[16];
            for (int v = 1; v < kp.V; ++v) m = fmaxf(m, red[16 + v]);
            float e[4], sum = 0.f;
            for (int v = 0; v < kp.V; ++v) { e[v] = __expf(red[16 + v] - m); sum += e[v]; }
            for (int v = 0; v < kp.V; ++v) kp.val[(size_t)board * kp.V + v] = e[v] / sum;
        }
        __syncthreads();    // scratch is reused by the next board
    }
}

}  // namespace gznn
