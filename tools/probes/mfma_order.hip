// Probe: cycles per v_mfma_f32_16x16x32_bf16 for the split trunk's issue pattern (one wave per SIMD,
// 16 accumulators, 3 products per accumulator per k-step) in two orders:
//   chain  : the three products of one accumulator back to back (the trunk's source order)
//   rr     : round-robin, each accumulator's products 16 MFMAs apart
//   free   : the compiler's order
// Operands live in registers (no memory traffic).  Prints cycles per MFMA (s_memtime, wave 0).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int ORDER>
__global__ void __launch_bounds__(256) probe(const bf16x8* in, float* out, unsigned long long* cyc, int iters) {
    const int lane = threadIdx.x;
    bf16x8 a0 = in[lane], a1 = in[lane + 64], b[8], c[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { b[t] = in[lane + 128 + 64 * t]; c[t] = in[lane + 640 + 64 * t]; }
    f32x4 acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[i][t] = f32x4{0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (ORDER == 0) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const bf16x8 w = ct ? a1 : a0;
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, b[t], acc[ct][t], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, c[t], acc[ct][t], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c[t ^ 1], b[t], acc[ct][t], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
        } else {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const bf16x8 w = ct ? a1 : a0;
                        const bf16x8 x = r == 0 ? w : (r == 1 ? w : c[t ^ 1]);
                        const bf16x8 y = r == 0 ? b[t] : (r == 1 ? c[t] : b[t]);
                        acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[ct][t], 0, 0, 0);
                        if (ORDER == 1) __builtin_amdgcn_sched_barrier(0);
                    }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) s += acc[i][t][0] + acc[i][t][1] + acc[i][t][2] + acc[i][t][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int iters = 2000, grid = 256;
    bf16x8* in;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&in, 2048 * sizeof(bf16x8));
    hipMemset(in, 0x3c, 2048 * sizeof(bf16x8));
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&cyc, grid * 8);
    unsigned long long h[256];
    for (int order = 0; order < 3; ++order) {
        for (int rep = 0; rep < 3; ++rep) {
            if (order == 0) probe<0><<<grid, 256>>>(in, out, cyc, iters);
            else if (order == 1) probe<1><<<grid, 256>>>(in, out, cyc, iters);
            else probe<2><<<grid, 256>>>(in, out, cyc, iters);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < grid; ++i) s += h[i];
        printf("%s: %.2f cycles per MFMA (mean over %d workgroups)\n", order == 0 ? "chain (3 dependent in a row)" : order == 1 ? "round-robin (distance 16)" : "compiler order",
               s / grid / (iters * 48.0), grid);
    }
    return 0;
}
