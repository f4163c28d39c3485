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
constexpr int kMaxSegments = 32;

// One contiguous run of boards of a launch: its planes and outputs may live anywhere the device
// can address (HBM, or pinned host memory of a game pool: zero-copy gather / scatter).
struct Segment {
    int row0;                      // first board of the segment within the launch
    const float* planes;           // [rows][C][H][W]
    float* pol[kMaxRoles];         // [rows][P_r]
    float* val;                    // [rows][V]
};

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct KParams {
    const __bf16* w0;        // initial conv, packed [K0/32][F][32]
    const float* b0;         // [F]
    const __bf16* wres;      // trunk convs, packed [2B][9][F/32][F][32]
    const float* bres;       // [2B][F]
    const float* wh;         // head 1x1 convs (BN folded) [2R+1][F]
    const float* bh;         // [2R+1]
    const float* pd[kMaxRoles];   // policy dense, transposed [P_r][2HW]
    const float* pb[kMaxRoles];   // [P_r]
    const float* vhw;        // value hidden, transposed [VH][HW]
    const float* vhb;        // [VH]
    const float* vdw;        // value dense [VH][V]
    const float* vdb;        // [V]
    int n;                   // boards in this launch
    int nseg;                // segments (>= 1), ascending row0, seg[0].row0 == 0
    Segment seg[kMaxSegments];
    unsigned long long* stamps;   // diagnostics only (GZ_KERNEL_STAMPS): [grid][8] s_memtime per phase
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

__device__ __forceinline__ int find_segment(const KParams& kp, int board) {
    int s = 0;
    while (s + 1 < kp.nseg && board >= kp.seg[s + 1].row0) ++s;
    return s;
}

// out[j] = bias[j] + sum_i WT[j][i] * x[i] for j < rows (x in LDS, WT row-major in global, fp32):
// 16 lanes per output row, 4 rows per wave, so every load instruction reads four 64-byte runs and
// each row's partial sums meet in a 4-step shuffle.  U row groups are in flight per wave at once:
// the loads of a group are independent, and issuing U*K/16 of them back to back turns U L2 round
// trips into one.
template <int K, int NWAVES>
__device__ __forceinline__ void dense_rows(const float* __restrict__ WT, const float* __restrict__ bias, int rows,
                                           const float* __restrict__ x, float* __restrict__ out, int wave, int lane) {
    constexpr int U = K <= 64 ? 8 : 4;
    constexpr int NI = (K + 15) / 16;
    const int l16 = lane & 15, sub = lane >> 4;
    float xv[NI];
#pragma unroll
    for (int n = 0; n < NI; ++n) xv[n] = (l16 + 16 * n < K) ? x[l16 + 16 * n] : 0.f;
    for (int j0 = 4 * wave + sub; j0 < rows; j0 += 4 * NWAVES * U) {
        float s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * 4 * NWAVES;
            const float* wr = WT + (size_t)(j < rows ? j : 0) * K;
            s[u] = 0.f;
#pragma unroll
            for (int n = 0; n < NI; ++n)
                if (l16 + 16 * n < K) s[u] += wr[l16 + 16 * n] * xv[n];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float v = s[u];
            v += __shfl_xor(v, 8, 64);
            v += __shfl_xor(v, 4, 64);
            v += __shfl_xor(v, 2, 64);
            v += __shfl_xor(v, 1, 64);
            const int j = j0 + u * 4 * NWAVES;
            if (l16 == 0 && j < rows) out[j] = v + bias[j];
        }
    }
}

// Weight prefetch that the compiler cannot move: issued as inline asm at the top of an iteration
// and consumed after an explicit vmcnt(0) at its end.  (Plain loads get sunk past the loop back
// edge to right before their first MFMA, which exposes the whole L2 latency every iteration.)
// The compiler does not track these loads, so gload_wait_all must precede any use of the result;
// gload_ready then re-defines each register after the wait so no copy can be hoisted above it.
__device__ __forceinline__ bf16x8 gload_issue(const __bf16* p) {
    bf16x8 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void gload_wait_all(bf16x8& v) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(v)::"memory"); }
__device__ __forceinline__ void gload_ready(bf16x8& v) { asm volatile("" : "+v"(v)); }

// One 3x3 'same' conv over the NB LDS images at X (board b at X + b*ACT_BYTES):
// acc[ct][t] = W * X (fp32 accumulate), tile t = b*PT + pt.  Every weight fragment loaded from L2
// feeds TT = NB*PT MFMAs -- NB is the weight-reuse factor that sets the L2->CU byte rate.
template <int F, int H, int W, int NB>
__device__ __forceinline__ void conv3x3(const char* __restrict__ X, const __bf16* __restrict__ wp,
                                        f32x4 (&acc)[Geo<F, H, W>::CT][Geo<F, H, W, NB>::TT],
                                        int co_base, int li, int g) {
    using G = Geo<F, H, W, NB>;
    constexpr int CT = G::CT, PT = G::PT, TT = G::TT, KC = G::KC;
    // The k loop runs as 9*KC/KS rolled iterations of KS k-steps (KS | KC, a tap or part of one).
    // Each iteration first issues the weight fragments of the NEXT iteration (one full iteration
    // of MFMAs hides their L2 latency), and double-buffers the activation fragments from LDS one
    // k-step ahead.  A rolled loop keeps the LDS address math out of registers.
    constexpr int KS = KC < 4 ? KC : 4;
    constexpr int NIT = 9 * KC / KS;
    static_assert(KC % KS == 0, "k-steps per iteration must divide the k-steps per tap");
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // lane's fragment of step s = tap*KC + kc: wp + ((s*F + co_base + 16ct + li) * 32 + 8g)
    const __bf16* wl = wp + (size_t)(co_base + li) * 32 + 8 * g;
    bf16x8 cur[KS][CT];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
            cur[k][ct] = *(const bf16x8*)(wl + ((size_t)k * F + 16 * ct) * 32);
    // land the first fragments before the loop so the loop header carries no pending loads
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) gload_ready(cur[k][ct]);

#pragma unroll 1
    for (int it = 0; it < NIT; ++it) {
        const int itn = it + 1 < NIT ? it + 1 : it;     // the last iteration re-reads its own
        bf16x8 nxt[KS][CT];
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                nxt[k][ct] = gload_issue(wl + ((size_t)(itn * KS + k) * F + 16 * ct) * 32);

        const int s0 = it * KS;
        const int tap = s0 / KC, kc0 = s0 % KC;
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
        bf16x8 b[2][TT];
        auto load_b = [&](int kc, bf16x8 (&dst)[TT]) {
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int off = qoff[pt] + (((kc * 4 + g) ^ qswz[pt]) << 4);
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) dst[bb * PT + pt] = *(const bf16x8*)(X + bb * G::ACT_BYTES + off);
            }
        };
        load_b(kc0, b[0]);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            if (k + 1 < KS) load_b(kc0 + k + 1, b[(k + 1) & 1]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int t = 0; t < TT; ++t)
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[k][ct], b[k & 1][t], acc[ct][t], 0, 0, 0);
        }
        // the prefetched fragments have had a whole iteration to land
        gload_wait_all(nxt[0][0]);
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                gload_ready(nxt[k][ct]);
                cur[k][ct] = nxt[k][ct];
            }
    }
}

// NB boards per workgroup of 4 waves; WPE = minimum resident waves per SIMD the register
// allocation must allow (amdgpu_waves_per_eu), i.e. WPE workgroups per CU.
template <int F, int H, int W, int NB, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
forward_kernel(const KParams kp) {
    using G = Geo<F, H, W, NB>;
    constexpr int NPOS = G::NPOS, PT = G::PT, TT = G::TT, CT = G::CT, kThreads = 256;
    constexpr int ACT = G::ACT_BYTES;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* X0 = smem;                 // [NB][ACT]
    char* X1 = smem + NB * ACT;      // [NB][ACT]
    char* SCR = X1;                  // scratch aliases X1 while X1 holds no live activations

    const int board0 = blockIdx.x * NB;
    const int tid = threadIdx.x;
#define GZ_STAMP(i) \
    if (kp.stamps && tid == 0) kp.stamps[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime()
    GZ_STAMP(0);
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
        const int sg = find_segment(kp, board0 + bb);
        const float* in = kp.seg[sg].planes + (size_t)(board0 + bb - kp.seg[sg].row0) * C * NPOS;
        for (int i = tid; i < C * NPOS; i += kThreads) sin[i] = live ? in[i] : 0.f;
        __syncthreads();
        // IM[p][k], k = tap*C + c, zero padded to K0: zero the image, then one thread per
        // (position, tap) copies its C channels (compile-time divisors only)
        for (int i = tid; i < (NPOS + 1) * K0 / 8; i += kThreads) ((uint4*)IM)[i] = uint4{0u, 0u, 0u, 0u};
        __syncthreads();
        for (int i = tid; i < NPOS * 9; i += kThreads) {
            const int p = i / 9, tap = i - (i / 9) * 9;
            const int y = p / W + tap / 3 - 1, x = p % W + tap % 3 - 1;
            if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
                const float* src = sin + y * W + x;
                for (int c = 0; c < C; ++c) {
                    const int k = tap * C + c;
                    *(__bf16*)(IM + p * imrow + ((((k >> 3) ^ (p & imswz))) << 4) + (k & 7) * 2) = (__bf16)src[c * NPOS];
                }
            }
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

    GZ_STAMP(1);
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

    GZ_STAMP(2);
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
        const int sg = find_segment(kp, board);
        const int row = board - kp.seg[sg].row0;
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
        if (bb == 0) GZ_STAMP(3);

        // policy heads: Dense(2HW -> P_r) + softmax
        for (int r = 0; r < kp.R; ++r) {
            const int P = kp.P[r];
            const float* pf = feat + r * 2 * NPOS;
            const float* wd = kp.pd[r];
            dense_rows<2 * NPOS, 4>(wd, kp.pb[r], P, pf, lg, wave, lane);
            __syncthreads();
            float lmax = -3.0e38f;
            for (int j = tid; j < P; j += kThreads) lmax = fmaxf(lmax, lg[j]);
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
                float* out = kp.seg[sg].pol[r] + (size_t)row * P;
                for (int j = tid; j < P; j += kThreads) out[j] = lg[j] * inv;
            }
            __syncthreads();
        }

        if (bb == 0) GZ_STAMP(4);
        // value head: Dense(HW -> VH) + act, Dense(VH -> V) + softmax
        const float* vf = feat + 2 * kp.R * NPOS;
        dense_rows<NPOS, 4>(kp.vhw, kp.vhb, kp.VH, vf, lg, wave, lane);
        __syncthreads();
        for (int k = tid; k < kp.VH; k += kThreads) lg[k] = act_fn(lg[k], kp.leaky);
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
            for (int v = 0; v < kp.V; ++v) kp.seg[sg].val[(size_t)row * kp.V + v] = e[v] / sum;
        }
        __syncthreads();    // scratch is reused by the next board
    }
    GZ_STAMP(5);
#undef GZ_STAMP
}

}  // namespace gznn
