// Forward of the residual policy/value CNN (v1, and v2 pre-activation with squeeze-excite and the
// global-pooling value head) for gfx950 (MI355X).
//
// trunk_kernel: one workgroup (4 waves; trunk_kernel8: two groups of 4 waves, a board each) takes
// NB boards through the whole network:
//   planes (fp32 NCHW, HBM staging or pinned host) -> im2col in LDS -> initial conv -> B residual
//   blocks -> the heads' 1x1 convs (+ the trunk's per-channel means for a pooling value head) ->
//   the dense policy / value heads + softmax, written straight to the callers' buffers (segments).
//   Trunk activations never leave the CU: the bf16 (hi + lo in split precision) copy that feeds the
//   next conv lives in LDS (two ping-pong images per board), the fp32 residual stream lives in
//   registers.
// Single-image kernels (F = 256 on 10 x 10 / 13 x 13: one image overwritten in place) write the head
// features to a device scratch instead; heads_kernel (and policy_gemm_kernel for large policies)
// then applies the dense heads.
//
// Each 3x3 conv is an implicit GEMM  out[co][p] = sum_{tap,ci} W[co][tap,ci] * X[nbr(p,tap)][ci]
// on v_mfma_f32_16x16x32_bf16, A = weights (rows co), B = activations (cols = positions).  Wave w
// owns output channels [w*F/4, (w+1)*F/4) for every position of the NB boards, so one weight
// fragment feeds NB*ceil(HW/16) MFMAs.
//
// Weight stream: every trunk conv's weights (bf16, BN folded, MFMA-fragment order) are one
// contiguous stream that each wave walks in "stages" of KS k-steps.  Stages land in a ring of R
// register slots, issued R-1 stages ahead by inline-asm loads the compiler cannot sink and counted
// with explicit s_waitcnt vmcnt(N): the ring runs continuously across conv boundaries and is primed
// before the input stage, so the L2/Infinity-Cache latency of the weight stream (~1 us when every
// CU streams) is covered by R-1 stages of MFMA work instead of one.
//
// LDS images: row q (a board position, plus one all-zero row) is ROWS = 512 bytes and holds the F
// bf16 channels as 16-byte chunks, logical chunk L at physical chunk L + s(q), s(q) = 2q mod 16
// (a rotation without wrap-around: the row has room for chunks 0 .. F/8+13).  The 4-bank group of
// a chunk is its index mod 16, so the two k-slices a ds_read_b128 lane group pairs (g, g^1) land on
// opposite parities and the 16 lanes of a group hit 16 distinct bank groups for every 3x3 shift;
// out-of-board neighbours read the zero row at the chunk of their virtual (unclipped) position,
// which keeps them conflict-free too.  Because the rotation adds, the k-steps of one tap differ by
// a constant byte offset: one address register per (tap, position tile) serves all of them.
//
// Reference semantics: src/ggpzero/nn/model.py:25-75, 154-296 (see oracle/nn_ref.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace gznn {

constexpr int kMaxRoles = 4;
constexpr int kMaxSegments = 32;
constexpr int kHeadBoards = 4;     // boards per heads_kernel workgroup (one softmax wave per board)
constexpr int kMaxSE = 64;         // squeeze-excite units

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
    const __bf16* w0;        // initial conv, packed [K0/32][F][32] (split precision: the hi parts)
    const __bf16* w0lo;      // split precision: the lo parts, same layout
    const float* b0;         // [F]
    const __bf16* wres;      // trunk convs, packed [2B][9][F/32][F][32] (split: [..][F][hi 32 | lo 32])
    const float* bres;       // [2B][F]
    const float* wh;         // head 1x1 convs (BN folded) [2R+1][F]
    const float* bh;         // [2R+1]
    const float* pd[kMaxRoles];   // policy dense, Keras layout [2HW][P_r] (k-major)
    const float* pb[kMaxRoles];   // [P_r]
    const float* vhw;        // value hidden, Keras layout [HW][VH]
    const float* vhb;        // [VH]
    const float* vdw;        // value dense [VH][V]
    const float* vdb;        // [V]
    // v2 (pre-activation) blocks, model.py:78-151
    const float* pre;        // [B][2][F]: BN before each block's first conv, as scale / shift
    const float* sew1;       // squeeze-excite compress [B][F][S] (Keras [in][out], padded channels 0)
    const float* sew2;       // squeeze-excite gating [B][S][F]
    float* feat;             // scratch [n][FS]: head features in flatten order (trunk -> heads)
    f32x4* resid;            // global-residual variants only: [grid][4 waves][CT*TT][64 lanes]
    int n;                  // boards in this launch
    int nseg;                // segments (>= 1), ascending row0, seg[0].row0 == 0
    Segment seg[kMaxSegments];
    unsigned long long* stamps;   // diagnostics only (GZ_KERNEL_STAMPS): [grid][8] s_memtime per phase
    int C, K0, B, R, VH, V, leaky, flatten_nchw, maxP, npos;
    int lgrow;               // floats per board of the dense heads' LDS outputs (heads_row)
    int heads_seq;           // dense heads one Dense after another (the two-phase row does not fit the LDS)
    int H, W, wmagic;        // board rows / columns; wmagic = ceil(65536 / W) (Board::div)
    int value_sigmoid;       // legacy model files: independent sigmoid per value output
    int logits;              // diagnostics (gz_net_set_output_logits): write pre-softmax / pre-sigmoid outputs
    // policy heads as an MFMA GEMM (single-image nets with large policies, policy_gemm_kernel):
    // packed weights [jt][kt][hi | lo][64 lanes][8] bf16 per role, logits scratch [n][sum P_r]
    int gemm_heads;
    const __bf16* pdp[kMaxRoles];
    int pkt;                 // k-tiles of 32 per role (2HW padded)
    float* glog;             // logits scratch
    int plog;                // sum of P_r (row stride of glog)
    int v2;                  // pre-activation blocks: stream s += conv2(act(BN(conv1(act(BN(s)))))) [* SE gate]
    int k0taps;              // initial conv taps: 9 (3x3) or 1 (1x1, v2)
    int init_act;            // activation after the initial conv (0: v2 files with a bare initial conv)
    int S;                   // squeeze-excite units (0: none), <= kMaxSE
    int gapF;                // pooling value head: the model's F channel means precede the value conv
    int FS;                  // head features per board: 2R*npos (policy) + gapF + npos (value)
    int btab_off;            // LDS byte offset of the trunk bias table
    int se_off;              // LDS byte offset of the squeeze-excite scratch
    int P[kMaxRoles];
    int VK;                  // value hidden Dense inputs per board: gapF + npos, or cal * npos
    // concat_all_layers value head (v2, model.py:251-260): cal = B + 1 trunk layers, each through a
    // 1x1 conv (BN folded: wcl [cal][F], bcl [cal]) + act; the trunk writes those features to the
    // device scratch as it goes and the dense heads run in heads_kernel (nofuse)
    int cal;
    const float* wcl;
    const float* bcl;
    int cal_off;             // LDS byte offset of the per-wave partial sums [4][NB][npos]
    int nofuse;              // two-image kernels: features to the device scratch, no fused heads
};

__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }

// the dense policy / value heads (defined with heads_kernel below; the two-image trunk kernels call
// it themselves)
template <int BPW, int NT = 256>
__device__ __forceinline__ void dense_heads(const KParams& kp, const float* fk, float* lg, int board0, int nb);

// The board geometry at run time (kernels are compiled per filter count and position-tile count):
// p / W as (p * ceil(65536 / W)) >> 16, exact for W <= 32 and p < 1024 (checked on the host).
constexpr int kMaxPTN = 23;        // position tiles of the largest compiled board (19 x 19)
struct Board {
    int H, W, npos, wmagic;
    // per lane and position tile pt (position p = 16 pt + lane % 16): bit tap (0-8) says whether p
    // is on the board and its neighbour at that 3x3 tap exists (set once per kernel), so a conv's
    // per-tap B-fragment addresses need no division, multiply or divergent bounds check
    int tapmask[kMaxPTN];
    __device__ __forceinline__ int row(int p) const { return (p * wmagic) >> 16; }
};

// Single-image kernels with the looped conv (deeper ring, single-buffered B fragments): measured
// slower than their fully unrolled conv on MI355X (cfg4 12.9 -> 14.6 ms, cfg5 equal at 1,024 rows,
// bit-identical; profiles/r04e_kexp.txt), so off; kept for experiments (tools/kexp siloop)
constexpr bool kLoopSI = false;
// Two-pass split (P = 2): the epilogues write each value's lo parts straight to the workgroup's lo
// scratch and its hi parts into the image, in one pass (instead of lo parts into the image, a
// copy-out sweep, then the hi parts)
constexpr bool kLoDirect = true;
// Two-image v1 kernels: each conv's epilogue inside its last k-step (conv3x3_looped EPI).  Measured
// no faster (bit-identical; residual trunk 490.7 k vs 489.4 k cycles per workgroup,
// profiles/r04z_epilogue_in_conv_kexp.txt): with one wave per SIMD the epilogue's VALU work issues in
// order between the MFMA chains and outlasts their shadow, so off; kept for experiments (kexp epioff)
constexpr bool kEpiInConv = false;

// Split two-image kernels' epilogue stores (store_act): one 16-byte store per lane after a lane swap
// instead of two 8-byte stores (whose 16 positions per store at the 544-byte row stride share banks
// two ways).  Bit-identical but no faster (profiles/r04za_store_swap_kexp.txt: 0.543-0.547 against
// 0.547-0.549 ms per 1,024-row launch, residual blocks 79.3 against 78.4 us): the stores are off the
// critical path, so off; kept for experiments (kexp swapon)
#ifndef GZ_STORE_SWAP
#define GZ_STORE_SWAP 0
#endif
constexpr bool kStoreSwap = GZ_STORE_SWAP != 0;

// variant 23's weight ring: one tap of stages (128 VGPRs) by default; 96 gives a 2-stage ring
// (experiments: -DGZ_H2_RING_VGPRS=96)
#ifndef GZ_H2_RING_VGPRS
#define GZ_H2_RING_VGPRS 128
#endif

// ring depth: largest R dividing the stages per conv with R slots of KS*CT fragments <= cap VGPRs
__host__ __device__ constexpr int ring_depth(int nst, int ks, int ct, int cap) {
    const int cand[5] = {9, 6, 4, 3, 2};
    for (int i = 0; i < 5; ++i)
        if (nst % cand[i] == 0 && cand[i] * ks * ct * 4 <= cap && (cand[i] - 1) * ks * ct <= 60) return cand[i];
    return 1;
}

__host__ __device__ constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }
__host__ __device__ constexpr int lcm_c(int a, int b) { return a / gcd_c(a, b) * b; }

// P = 1: bf16 operands.  P = 3: split precision ("fp32 accuracy"): every fp32 operand x is carried
// as x_hi = bf16(x), x_lo = bf16(x - x_hi) and each product as hi*hi + hi*lo + lo*hi (three MFMAs,
// fp32 accumulation): ~16 significant bits per operand instead of 8.
// P = 2: the same split products for single-image kernels whose hi + lo image exceeds the LDS
// (F = 256 on 13 x 13): the LDS image holds one part at a time.  Each conv runs two passes over the
// same weight stages: pass 0 over the hi image (W_hi x_hi + W_lo x_hi), then the lo image is copied
// in from a per-workgroup device scratch (written by the previous epilogue) and pass 1 adds
// W_hi x_lo.
// WG = wave groups per workgroup: 1 (4 waves for NB boards) or 2 (8 waves, 2 per SIMD: group g takes
// board g of the workgroup with NB = 1; the register budget is then 256 per wave); WG = 3: ONE group
// of 8 waves for the NB boards, each wave a half of the 4-wave layout's output channels (CT halves:
// the same weight stream per workgroup, two waves per SIMD, 256 registers per wave); WG = 4: two
// groups of 2 waves, a board each (NB = 1), each wave half the output channels of its board (twice
// the 4-wave layout's co tiles, half its position tiles: half the B-fragment reads per MFMA, twice
// the weight fragments)
template <int F, int PTN, int NB = 1, int P = 1, int WG = 1>
struct Geo {
    static constexpr int P2 = P == 3 ? 2 : 1;        // bf16 parts per activation in the LDS image
    static constexpr int WP = P == 1 ? 1 : 2;        // bf16 parts per weight
    // the board (H x W, runtime: kp.H / kp.W) has at most NPOS = 16 * PTN positions
    static constexpr int NPOS = 16 * PTN;            // position capacity (the real count is kp.npos)
    static constexpr int PT = PTN;                   // position tiles per board (MFMA N)
    static constexpr int TT = NB * PT;               // position tiles per wave (all boards)
    static constexpr int NWV = WG == 3 ? 8 : WG == 4 ? 2 : 4;   // waves per group
    static constexpr int NGR = WG == 2 || WG == 4 ? 2 : 1;      // wave groups per workgroup
    static constexpr int CT = F / (16 * NWV);        // co tiles per wave (MFMA M)
    static constexpr int KC = F / 32;                // k-steps per tap
    static constexpr int CPR = F / 8;                // 16-byte chunks of channels per row
    // Split precision with F = 128 (16 chunks, 256 B per part): the rotation wraps inside the
    // 256-byte row (WRAP), so hi + lo fit 512 bytes and two boards fit a workgroup's LDS (k-step
    // offsets then need an add + and per read: measured slower for the bf16 kernels, which keep
    // rows with room for the rotated chunks without wrap-around, profiles/r02h_kernel_variants_*)
    // (F = 256 split, single image: the same wrapped rotation inside 512-byte rows, so the hi + lo
    // image of a 10 x 10 board fits the LDS)
    //
    // Padded rows (WRAP, the split kernels with >= 16 chunks per part): the rotation is replaced by
    // a 32-byte pad per row -- row q, chunk c at byte q * ROWS + 16 c with ROWS = 2 * 16 CPR + 32,
    // whose 16-byte bank group (34 q + c) mod 16 = (2 q + c) mod 16 is the rotated layout's --
    // so a k-step's B reads differ by immediate offsets again (no add + and per read).  Off-board
    // neighbours read a zero area (two rows) at the rotated chunk of their virtual position.
    // Large boards (more than 11 position tiles, up to 19 x 19: one part per row, two-pass split)
    // take the same padded rows for their single part: ROWS = 16 CPR + 32, bank group
    // (18 q + c) mod 16 = (2 q + c) mod 16 again (F = 128: 288 bytes a row, the 19 x 19 image 107 KB,
    // where the rotated 512-byte rows would need 190 KB)
    static constexpr bool WRAP = CPR >= 16 && (P2 == 2 || PTN > 11);
    static constexpr int HALF = WRAP ? CPR * 16 : ((CPR + 14) * 16 + 255) & ~255;   // one part's row
    static constexpr int ROWS = WRAP ? P2 * HALF + 32 : P2 * HALF;   // LDS row stride: hi part, then lo part
    static constexpr int ZROWS = WRAP ? 2 : 1;       // zero rows (padded rows: reads up to ROWS + 512)
    // + the all-zero row(s) (from row kp.npos: every off-board 3x3 neighbour reads there) and one
    // scratch row (row kp.npos + ZROWS: the epilogues of a partial last position tile store their
    // off-board lanes there instead of branching around the store)
    static constexpr int ACT_BYTES = (NPOS + ZROWS + 1) * ROWS;
    // k-steps per ring stage and the ring's VGPR budget: F = 256 (4 co tiles per wave, 16 weight
    // VGPRs per k-step) streams single k-steps through a 64-VGPR ring so the accumulators, the
    // residual and the B fragments still fit the 512 registers of a wave without spilling
    static constexpr int KS = (CT >= 4 || WP == 2) ? 1 : 2;
    static constexpr int NFR = CT * WP;              // weight fragments per k-step per lane
    static constexpr int ROWB = 64 * WP;             // bytes per output channel per k-step
    static constexpr int NST = 9 * KC / KS;          // ring stages per conv
    // ring depth; the two-board split kernels take exactly one tap's stages (R = KC / KS) so the
    // looped conv's body is one tap (a deeper ring made the body three taps and spilled)
    static constexpr int R0 = (P2 == 2 && (NB == 2 || WG == 2 || WG == 4) && (KC / KS) >= 3 && NST % (KC / KS) == 0 &&
                               (KC / KS) * KS * NFR * 4 <= (WG == 4 ? GZ_H2_RING_VGPRS : 96))
                                  ? KC / KS
                                  : ring_depth(NST, KS, NFR, CT >= 4 ? 64 : 96);
    // Single-image mode: when two ping-pong images (+ bias table) do not fit the 160 KB of LDS
    // (F = 256 on 10x10 / 13x13 boards), or the registers are nearly full anyway (large boards:
    // the single-image epilogue keeps fewer values live), one image is overwritten in place: every conv's MFMAs
    // finish reading it (barrier) before its epilogue writes it.  The input staging and head
    // scratch then alias the image.
    // live VGPRs of the trunk loop: weight ring + double-buffered B fragments + accumulators +
    // residual stream
    static constexpr int LIVE_VGPRS = R0 * KS * NFR * 4 + 2 * TT * P2 * 4 + 2 * CT * TT * 4;
    // (the two-pass split kernels, P = 2, are single-image by construction)
    static constexpr bool SI = 2 * NB * ACT_BYTES + 16 * 1024 > 160 * 1024 || (NB == 1 && LIVE_VGPRS > 330) || P == 2;
    // ring depth: single-image kernels run the looped conv (single-buffered B fragments), which
    // leaves room for a deeper ring (up to 128 VGPRs: F = 256 split, 4 stages = 3 k-steps ahead of
    // the MFMAs; its weights stream from the MALL, not the L2)
    static constexpr int RS = ring_depth(NST, KS, NFR, 64);
    static constexpr int US = lcm_c(RS, KC / KS) * ((lcm_c(RS, KC / KS) * KS) % 2 ? 2 : 1);
    // (large boards always loop: the unrolled conv's double-buffered B fragments alone would take
    // 2 x 23 x 4 VGPRs beside 184 accumulators)
    static constexpr bool LOOPSI = (kLoopSI || PTN > 11) && SI && NST % US == 0 && NST / US >= 2;
    static constexpr int R = LOOPSI ? RS : R0;
    static constexpr int LPS = KS * NFR;             // weight loads per stage per lane
    // Global residual: when the fp32 residual stream (+ the accumulators) would need more than 256
    // VGPRs (F = 256 on 13x13: 2 x 176), it lives in a per-workgroup device scratch instead of
    // registers, lane-contiguous (one coalesced 1 KB store / load per wave and tile).
    static constexpr bool RG = CT * TT * 4 * 2 > 256;
    // Compiler-tracked weight loads: above ~300 live VGPRs (ring + double-buffered B fragments +
    // accumulators + residual) the register allocator moves values between VGPRs and AGPRs, and a
    // copy of an inline-asm load's destination could be taken before the data lands; such kernels
    // (and the single-image ones) issue the ring with ordinary loads, which the compiler waits for.
    static constexpr bool TRACKED = SI || LIVE_VGPRS > 300 || (P2 == 2 && (NB == 2 || WG == 2 || WG == 4));
    static_assert(F % 64 == 0, "filters must be a multiple of 64");
    static_assert(!SI || NB == 1, "single-image mode takes one board per workgroup");
    static_assert(WG == 1 || ((WG == 2 || WG == 4) && NB == 1 && !SI) || (WG == 3 && !SI && CT >= 1), "wave groups: two images");
    static_assert(!RG || SI, "the global residual is implemented for single-image kernels");
    static constexpr int RESID_BYTES = RG ? 4 * CT * TT * 64 * 16 : 0;   // per workgroup
    // P = 2: the lo image of each workgroup (device scratch after the grid's residual scratch)
    static constexpr int LO_BYTES = P == 2 ? ACT_BYTES : 0;
    static_assert(KC % KS == 0, "a stage must not straddle a tap");
    static_assert(R >= 2, "no ring depth fits");
    // Looped conv (two-image kernels): the 9-tap conv runs as NIT iterations of a body of U ring
    // stages (a whole number of ring slots and of taps, an even number of k-steps so the B
    // double buffer's parity is static) instead of fully unrolled: the unrolled conv pair of a
    // residual block was ~100 KB of code, far beyond the instruction cache, so every block
    // re-streamed its instructions (measured 21 cycles per MFMA with every memory access removed,
    // against 16.5 for a register-only MFMA loop; profiles/r03bc_*).
    static constexpr int SPT = KC / KS;                                  // ring stages per tap
    static constexpr int U0 = lcm_c(R, SPT);
    static constexpr int U = (U0 * KS) % 2 ? 2 * U0 : U0;                // stages per iteration
    static constexpr int NIT = NST / U;
    static constexpr int TPI = U * KS / KC;                              // taps per iteration
    static constexpr bool LOOP = !SI && NST % U == 0 && NIT >= 2;
    static_assert(!LOOPSI || (NST % U == 0 && NIT >= 2), "single-image looped conv");
};

// chunk rotation of LDS row q (q may be a virtual, off-board position)
__device__ __forceinline__ int swz(int q) { return (2 * q) & 14; }

// LDS bytes of the trunk kernel beyond the two activation image sets: bias table + scratch
// (input staging / 1x1-head partials; the scratch aliases the second image set).
__host__ __device__ inline int trunk_scratch_bytes(int npos, int C, int K0, int R, int P2, int F) {
    const int in_stage = align16(C * npos * 4) + P2 * align16((npos + 1) * K0 * 2);
    const int hc = 2 * R + 1;
    const int heads = align16((F / 16) * hc * npos * 4);   // head-conv partials per 16-channel tile
    return in_stage > heads ? in_stage : heads;
}
__host__ __device__ inline int bias_table_bytes(int F, int B) { return align16((2 * B) * F * 4); }
// squeeze-excite scratch: per board the channel means [F] and the compressed units [kMaxSE]
__host__ __device__ inline int se_scratch_bytes(int F, int NB) { return NB * (F + kMaxSE) * 4; }

__device__ __forceinline__ float act_fn(float v, int leaky) {
    return v > 0.f ? v : (leaky ? 0.03f * v : 0.f);
}
// The same activation as max(v, alpha v), alpha = 0 (ReLU) or 0.03 (LeakyReLU), alpha < 1: a
// multiply and a max, no compare / select, for the two-image kernels' residual epilogues (a
// negative v gives -0.0 under ReLU instead of +0.0; no later use depends on the sign).  (In the
// single-image kernels this form raised register pressure: they keep act_fn.)
__device__ __forceinline__ float act_mx(float v, float alpha) { return fmaxf(v, alpha * v); }

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    __bf16 x = (__bf16)a, y = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

__device__ __forceinline__ float bf16_lo(float x) { return x - (float)(__bf16)x; }

// SEL: off-board lanes of a partial last tile write the scratch row (a select, not a branch: the
// two-image kernels); otherwise they branch around the store (single-image kernels, whose 40+ tile
// epilogues keep fewer values live that way).  P = 2: the lo parts (the epilogue's first image; the
// workgroup saves it to device memory and then writes the hi parts, save_lo_write_hi).
template <int F, int PTN, int P = 1, bool SEL = true>
__device__ __forceinline__ void store_act(char* X, int p, int co, f32x4 v, int npos) {
    using G = Geo<F, PTN, 1, P>;
    if constexpr (SEL && G::WRAP && kStoreSwap) {
        // Split two-image kernels: the lanes of rows 2r and 2r + 1 (channel groups g, g + 1 of one
        // position) trade halves with one v_permlane16_swap per dword, so row 2r holds the hi parts of
        // the 8 channels and row 2r + 1 their lo parts: one 16-byte store per lane (the chunk's hi
        // half, or its lo half at + HALF) instead of two 8-byte stores, the same bytes in the image.
        // (Every lane takes part: no branch around it.)
        const int q = p >= npos ? npos + G::ZROWS : p;
        const uint32_t h0 = pack2(v[0], v[1]), h1 = pack2(v[2], v[3]);
        const uint32_t l0 = pack2(bf16_lo(v[0]), bf16_lo(v[1])), l1 = pack2(bf16_lo(v[2]), bf16_lo(v[3]));
        const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
        char* a = X + q * G::ROWS + ((co >> 3) << 4) + ((co & 4) ? G::HALF : 0);
        *(uint4*)a = uint4{s0[0], s1[0], s0[1], s1[1]};
        return;
    }
    if (SEL || p < npos) {
        const int q = SEL && p >= npos ? npos + G::ZROWS : p;
        const int chunk = G::WRAP ? (co >> 3) : ((co >> 3) + swz(q));
        char* a = X + q * G::ROWS + (chunk << 4) + (co & 7) * 2;
        uint2 u;
        if constexpr (P == 2) {
            u.x = pack2(bf16_lo(v[0]), bf16_lo(v[1]));
            u.y = pack2(bf16_lo(v[2]), bf16_lo(v[3]));
        } else {
            u.x = pack2(v[0], v[1]);
            u.y = pack2(v[2], v[3]);
        }
        *(uint2*)a = u;
        if constexpr (G::P2 == 2) {    // the lo part, same chunk of the row's second half
            uint2 l;
            l.x = pack2(bf16_lo(v[0]), bf16_lo(v[1]));
            l.y = pack2(bf16_lo(v[2]), bf16_lo(v[3]));
            *(uint2*)(a + G::HALF) = l;
        }
    }
}

// P = 2 (kLoDirect): the lo parts of v straight to the workgroup's lo scratch, at the byte offset
// the image would hold them (on-board positions only)
template <int F, int PTN>
__device__ __forceinline__ void store_lo_scratch(char* xlo, int p, int co, f32x4 v, int npos) {
    using G = Geo<F, PTN, 1, 2>;
    if (p < npos) {
        const int chunk = G::WRAP ? (co >> 3) : (co >> 3) + swz(p);
        uint2 l;
        l.x = pack2(bf16_lo(v[0]), bf16_lo(v[1]));
        l.y = pack2(bf16_lo(v[2]), bf16_lo(v[3]));
        *(uint2*)(xlo + p * G::ROWS + (chunk << 4) + (co & 7) * 2) = l;
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

__device__ __forceinline__ int find_segment(const KParams& kp, int board) {
    int s = 0;
    while (s + 1 < kp.nseg && board >= kp.seg[s + 1].row0) ++s;
    return s;
}

// Weight-stream loads the compiler cannot move: issued as inline asm, consumed after an explicit
// s_waitcnt vmcnt(N).  The compiler does not track these loads, so ring_wait must precede any use
// of the result; ring_ready then re-defines each register after the wait so no use (or copy) can be
// hoisted above it.  Every issued register stays live until consumed or until ring_drain.
template <int IMM>
__device__ __forceinline__ bf16x8 gload_issue(uint32_t voff, const void* sbase) {
    bf16x8 v;
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(v) : "v"(voff), "s"(sbase), "n"(IMM) : "memory");
    return v;
}
template <int N>
__device__ __forceinline__ void ring_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void ring_ready(bf16x8& v) { asm volatile("" : "+v"(v)); }

// ---- trunk -------------------------------------------------------------------------------------

template <int F, int PTN, int NB, int P, int WG = 1>
struct Ring {
    using G = Geo<F, PTN, NB, P, WG>;
    bf16x8 r[G::R][G::KS][G::NFR];    // fragment f = ct * WP + part
};

// Issue stage `gs` of the trunk weight stream (clamped to the last stage) into ring slot SLOT.
// Fragment (step, ct, part) of a lane: wres + step*F*ROWB + (ct*WP + part)*1 KB + woff, woff = the
// wave's first 16-channel block + 16 bytes * lane (gz_nn.hip wres_index: each fragment is 1 KB in
// lane order, so a wave's load is one contiguous 1 KB); the stage base is scalar, the fragment's
// offset the instruction's immediate.
// Single-image (F = 256) kernels run at the 512-register limit, where the register allocator
// copies values between VGPRs and AGPRs freely: an inline-asm load's destination could be copied
// (or its register reused) before the data lands.  They issue the ring with ordinary loads, which
// the compiler tracks (it places the waits and never copies an in-flight register).
// byte offset of weight fragment f (= ct * WP + part) within a k-step, relative to the wave's first block
template <int WP, int ROWB, int FR>
struct FragOff {
    static_assert(ROWB == 64 * WP, "16 rows x ROWB bytes = WP fragments of 1 KB");
    static constexpr int value = FR * 1024;
};
template <int F, int PTN, int NB, int P, int WG, int SLOT, int PARTS, int FR>
__device__ __forceinline__ void ring_issue_f(Ring<F, PTN, NB, P, WG>& ring, int k, uint32_t woff, const char* sb) {
    using G = Geo<F, PTN, NB, P, WG>;
    if constexpr ((PARTS >> (FR % G::WP)) & 1) {
        if constexpr (G::TRACKED)
            ring.r[SLOT][k][FR] = *(const bf16x8*)(sb + woff + FragOff<G::WP, G::ROWB, FR>::value);
        else
            ring.r[SLOT][k][FR] = gload_issue<FragOff<G::WP, G::ROWB, FR>::value>(woff, sb);
    }
}
template <int F, int PTN, int NB, int P, int WG, int SLOT, int PARTS, int... FRS>
__device__ __forceinline__ void ring_issue_k(Ring<F, PTN, NB, P, WG>& ring, int k, uint32_t woff, const char* sb,
                                             std::integer_sequence<int, FRS...>) {
    (ring_issue_f<F, PTN, NB, P, WG, SLOT, PARTS, FRS>(ring, k, woff, sb), ...);
}
// PARTS: bit 0 the hi fragments, bit 1 the lo fragments.  P = 2: a stage of a conv's second pass
// multiplies by the hi parts only, so its lo fragments are not loaded (their slot registers are not
// read in that pass; TRACKED kernels only)
template <int F, int PTN, int NB, int P, int WG, int SLOT, int PARTS = 3>
__device__ __forceinline__ void ring_issue(Ring<F, PTN, NB, P, WG>& ring, const __bf16* wres, uint32_t woff, int gs, int gmax) {
    using G = Geo<F, PTN, NB, P, WG>;
    int s = gs < gmax ? gs : gmax;
    // P = 2: global stage gs runs pass gs / NST % 2 of conv gs / (2 NST); both passes stream the
    // conv's weight stages
    if constexpr (P == 2) s = (s / (2 * G::NST)) * G::NST + s % G::NST;
#pragma unroll
    for (int k = 0; k < G::KS; ++k)
        ring_issue_k<F, PTN, NB, P, WG, SLOT, PARTS>(ring, k, woff, (const char*)wres + (size_t)(s * G::KS + k) * F * G::ROWB,
                                                    std::make_integer_sequence<int, G::NFR>{});
}

// LDS byte offset (within a board image) of a lane's B fragment for tap `tap`, position tile pt,
// k-step 0 of the tap; k-step kc adds kc*64.  Callers launder `lane` (an empty asm redefinition)
// once per tap so these offsets are computed when the tap starts instead of being hoisted for all
// nine taps out of the trunk loop, which would pin 9*PT address registers for the whole kernel.
__device__ __forceinline__ void launder(int& v) { asm volatile("" : "+v"(v)); }
template <typename T>
__device__ __forceinline__ void launder_ptr(T*& p) { asm volatile("" : "+v"(p)); }
// A lane's B-fragment address for tap `tap`, tile pt: row base + rotated chunk offset of k-step 0.
// k-step kc reads chunk offset (rot + 64 kc), wrapped to the 256-byte row under WRAP (k-step
// offsets are then not immediates: one add + and per read).
struct TapAddr {
    int row, rot;
};
template <int F, int PTN, int P = 1>
__device__ __forceinline__ TapAddr tap_base(int tap, int pt, int lane, const Board& bd) {
    using G = Geo<F, PTN, 1, P>;
    const int li = lane & 15, g = lane >> 4;
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
    const int p = 16 * pt + li;
    static_assert(PTN <= kMaxPTN, "board larger than the tap masks");
    const int qv = p + (dy * bd.W + dx);                 // the (virtual) neighbour position
    const bool ok = (bd.tapmask[pt] >> tap) & 1;
    if constexpr (G::WRAP) {   // padded rows: chunk g of row qv, or the zero area at the rotated chunk
        const int a_in = qv * G::ROWS + (g << 4);
        const int a_zero = bd.npos * G::ROWS + (((g + swz(qv)) & 15) << 4);
        const int m = -(int)ok;    // both computed and masked: no divergent branch per tap and tile
        return TapAddr{(a_in & m) | (a_zero & ~m), 0};
    }
    const int rot = (g + swz(qv)) << 4;
    return TapAddr{(ok ? qv : bd.npos) * G::ROWS, rot};
}
template <int F, int PTN, int P = 1>
__device__ __forceinline__ int tap_offset(const TapAddr& t, int kc) {
    return t.row + t.rot + 64 * kc;
}

// One 3x3 'same' conv over the NB LDS images at X (board b at X + b*ACT_BYTES):
// acc[ct][t] = W * X (fp32 accumulate), tile t = b*PT + pt.  gs0 = global stage index of this
// conv's first stage; on entry stages gs0 .. gs0+R-2 are in flight in ring slots 0..R-2.
template <int F, int PTN, int NB, int P, int WG, int PASS, int ST>
__device__ __forceinline__ void conv_stage(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                           f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                           bf16x8 (&b)[2][Geo<F, PTN, NB, P, WG>::TT][Geo<F, PTN, NB, P, WG>::P2],
                                           const __bf16* wres, uint32_t woff, int gs0, int gmax, int& lane,
                                           const Board& bd) {
    using G = Geo<F, PTN, NB, P, WG>;
    constexpr int R = G::R, KS = G::KS, CT = G::CT, PT = G::PT, TT = G::TT, KC = G::KC, P2 = G::P2, WP = G::WP;
    // refill the slot stage ST-1 consumed with stage ST+R-1, then wait for stage ST
    // P = 2: the stage issued here belongs to this pass, or (past the pass's last stage) to the
    // next one; the second pass's stages need the hi parts only
    constexpr bool next_in_pass = ST + R - 1 < G::NST;
    constexpr bool hi_only = P == 2 && G::TRACKED && (next_in_pass ? PASS == 1 : PASS == 0);
    ring_issue<F, PTN, NB, P, WG, (ST + R - 1) % R, hi_only ? 1 : 3>(ring, wres, woff, gs0 + ST + R - 1, gmax);
    if constexpr (!G::TRACKED) {
        ring_wait<(R - 1) * G::LPS>();
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int f = 0; f < G::NFR; ++f) ring_ready(ring.r[ST % R][k][f]);
    }

#pragma unroll
    for (int k = 0; k < KS; ++k) {
        const int j = ST * KS + k;             // k-step within the conv
        if (j + 1 < 9 * KC) {                  // B fragments of the next k-step (double buffer)
            const int jn = j + 1;
            const int tap = jn / KC, kc = jn % KC;
            if (kc == 0) launder(lane);
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const char* a = X + tap_offset<F, PTN, P>(tap_base<F, PTN, P>(tap, pt, lane, bd), kc);
#pragma unroll
                for (int bb = 0; bb < NB; ++bb)
#pragma unroll
                    for (int h = 0; h < P2; ++h)
                        b[jn & 1][bb * PT + pt][h] = *(const bf16x8*)(a + bb * G::ACT_BYTES + h * G::HALF);
            }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const bf16x8 w_hi = ring.r[ST % R][k][ct * WP];
                acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[j & 1][t][0], acc[ct][t], 0, 0, 0);
                if constexpr (P == 3) {   // split precision: + hi*lo + lo*hi
                    const bf16x8 w_lo = ring.r[ST % R][k][ct * WP + 1];
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[j & 1][t][1], acc[ct][t], 0, 0, 0);
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[j & 1][t][0], acc[ct][t], 0, 0, 0);
                } else if constexpr (P == 2 && PASS == 0) {   // two-pass split, hi image: + lo*hi
                    const bf16x8 w_lo = ring.r[ST % R][k][ct * WP + 1];
                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[j & 1][t][0], acc[ct][t], 0, 0, 0);
                }   // (P = 2, pass 1: the lo image, hi*lo only)
            }
        // interleave the next k-step's B reads with this k-step's MFMAs (CT MFMAs, one ds_read,
        // ...) instead of the compiler's cluster of reads ahead of the MFMA run: measured 2-4 %
        // faster at 640-1024 rows, neutral at 256 (same-box A/B, profiles/r01l_interleave_ab.txt)
        if constexpr (!G::SI) {
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                __builtin_amdgcn_sched_group_barrier(0x008, CT * (P2 == 2 ? 3 : 1), 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, P2, 0);                       // DS read
            }
        }
        // k-step boundary: nothing crosses it, so the next k-step's B reads stay one k-step ahead
        // of their MFMAs (double buffer) and scheduling regions stay one k-step long (also in the
        // single-image kernels: without it their 9-tap branch-free conv became one region whose
        // schedule put each B read next to its use)
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int F, int PTN, int NB, int P, int WG, int... S>
__device__ __forceinline__ void ring_prime(Ring<F, PTN, NB, P, WG>& ring, const __bf16* wres, uint32_t woff, int gmax,
                                           std::integer_sequence<int, S...>) {
    (ring_issue<F, PTN, NB, P, WG, S>(ring, wres, woff, S, gmax), ...);
}

template <int F, int PTN, int NB, int P, int WG, int PASS, int... ST>
__device__ __forceinline__ void conv_stages(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                            f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                            bf16x8 (&b)[2][Geo<F, PTN, NB, P, WG>::TT][Geo<F, PTN, NB, P, WG>::P2],
                                            const __bf16* wres, uint32_t woff, int gs0, int gmax, int& lane,
                                            const Board& bd, std::integer_sequence<int, ST...>) {
    (conv_stage<F, PTN, NB, P, WG, PASS, ST>(X, ring, acc, b, wres, woff, gs0, gmax, lane, bd), ...);
}

// PASS (P = 2): 0 starts the accumulators, 1 adds to them
template <int F, int PTN, int NB, int P, int WG = 1, int PASS = 0>
__device__ __forceinline__ void conv3x3(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                        f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                        const __bf16* wres, uint32_t woff, int gs0, int gmax, int lane,
                                        const Board& bd) {
    using G = Geo<F, PTN, NB, P, WG>;
    constexpr int PT = G::PT, TT = G::TT;
    if constexpr (PASS == 0) {
#pragma unroll
        for (int ct = 0; ct < G::CT; ++ct)
#pragma unroll
            for (int t = 0; t < TT; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    bf16x8 b[2][TT][G::P2];
    // k-step 0 = tap 0 (dy = dx = -1), kc 0
    launder(lane);
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
        const char* a = X + tap_offset<F, PTN, P>(tap_base<F, PTN, P>(0, pt, lane, bd), 0);
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
#pragma unroll
            for (int h = 0; h < G::P2; ++h) b[0][bb * PT + pt][h] = *(const bf16x8*)(a + bb * G::ACT_BYTES + h * G::HALF);
    }
    conv_stages<F, PTN, NB, P, WG, PASS>(X, ring, acc, b, wres, woff, gs0, gmax, lane, bd,
                                     std::make_integer_sequence<int, G::NST>{});
}

// ---- looped conv: one iteration = U ring stages = TPI taps; tap0 = the iteration's first tap ----
// B fragments are single-buffered per tile: tile t's fragments for the next k-step are read right
// after tile t's last MFMA of this k-step (the other tiles' MFMAs, ~670 cycles, cover the LDS
// latency), which saves the 64 VGPRs of a second buffer; the register allocator otherwise shuffled
// loop-carried values between VGPRs and AGPRs every iteration.
// P = 2 (two-pass split, PASS 0 / 1; single-image kernels): pass 0 multiplies the hi image by the hi
// and lo weights, pass 1 the lo image by the hi weights only, so pass 1 loads no lo fragments -- except
// where a stage of the last iteration looks ahead into the next conv's pass 0 (and pass 0's look-ahead
// into pass 1 skips them): a uniform branch on last_it around those loads.
// The split product of one (co tile, position tile) in the looped conv -- hi*hi + hi*lo + lo*hi --
// as ONE inline-asm accumulate chain with dst == srcC.  With the builtins the register allocator
// renamed accumulators across the loop (dst != srcC, then VGPR / AGPR copies at the loop top); the
// chain keeps every accumulator in its AGPRs (-4 % launch time at 1,024 rows, bit-identical,
// profiles/r04e_kexp.txt).  Hazards (nothing inside an asm string is padded by the compiler): an
// MFMA taking the previous MFMA's D whole as C needs no wait states; the A/B operands come from
// LDS / global loads (no VALU write before the chain; tests/test_kernel_asm_audit.py checks the
// compiled kernels for copies into them or accesses to the accumulators inside the loop); the
// accumulators' zeroing and the epilogue's reads are fenced by split_chain_enter / _leave.
__device__ __forceinline__ void mfma_split3(f32x4& acc, const bf16x8& wh, const bf16x8& bh, const bf16x8& bl,
                                            const bf16x8& wl) {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %4, %2, %0"
        : "+a"(acc)
        : "v"(wh), "v"(bh), "v"(bl), "v"(wl));
}
// before the first chain: every accumulator is materialised (its zeroing, a VALU write) ahead of a
// 2-state pad (VALU write -> MFMA operand)
template <int CT, int TT>
__device__ __forceinline__ void split_chain_enter(f32x4 (&acc)[CT][TT]) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < TT; ++t) asm volatile("" : "+a"(acc[ct][t]));
    asm volatile("s_nop 1" ::: "memory");
}
// after the last chain: 24 states (an MFMA's D -> any other reader or writer: 12 for 8 passes, 19 for
// 16), then every accumulator redefined, so no read of one is scheduled above the pad
template <int CT, int TT>
__device__ __forceinline__ void split_chain_leave(f32x4 (&acc)[CT][TT]) {
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < TT; ++t) asm volatile("" : "+a"(acc[ct][t]));
}

// No epilogue inside the conv (the default)
struct NoEpi {
    __device__ __forceinline__ void operator()(int) const {}
};

// EPI (the conv's last iteration): the epilogue of position tile t - 1 runs right after tile t's MFMAs
// of the conv's final k-step (and tile TT - 1's after the last), so the epilogue's VALU work overlaps
// the remaining MFMAs instead of following them all.  Its reads of tile t - 1's accumulators come
// behind a 20-state pad pinned to them (MFMA D -> VALU read; split kernels' asm chains).  The
// epilogue writes the OTHER image (two-image kernels), which no wave reads in this conv.
template <int CT, int TT>
__device__ __forceinline__ void tile_leave(f32x4 (&acc)[CT][TT], int t) {
    asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) asm volatile("" : "+a"(acc[ct][t]));
}

template <int F, int PTN, int NB, int P, int WG, int PASS, int ST, bool EPI = false, class Epi = NoEpi>
__device__ __forceinline__ void conv_stage_l(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                             f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                             bf16x8 (&b)[Geo<F, PTN, NB, P, WG>::TT][Geo<F, PTN, NB, P, WG>::P2],
                                             const __bf16* wres, uint32_t woff, int gs_it, int gmax, int& lane,
                                             const Board& bd, int tap0, bool last_it, const Epi& epi = Epi{}) {
    using G = Geo<F, PTN, NB, P, WG>;
    constexpr int R = G::R, KS = G::KS, CT = G::CT, PT = G::PT, KC = G::KC, P2 = G::P2, WP = G::WP;
    static_assert(P != 2 || G::TRACKED, "two-pass split: compiler-tracked weight loads");
    static_assert(G::U % R == 0, "ring slots must be static within an iteration");
    if constexpr (P == 2) {
        constexpr int SLOT = (ST + R - 1) % R;
        const int gs = gs_it + ST + R - 1;
        ring_issue<F, PTN, NB, P, WG, SLOT, 1>(ring, wres, woff, gs, gmax);
        if constexpr (ST + R - 1 < G::U) {    // a stage of this iteration's pass
            if constexpr (PASS == 0) ring_issue<F, PTN, NB, P, WG, SLOT, 2>(ring, wres, woff, gs, gmax);
        } else if ((PASS == 0) != last_it) {  // the next iteration's, or the next pass's (last_it)
            ring_issue<F, PTN, NB, P, WG, SLOT, 2>(ring, wres, woff, gs, gmax);
        }
    } else {
        ring_issue<F, PTN, NB, P, WG, (ST + R - 1) % R>(ring, wres, woff, gs_it + ST + R - 1, gmax);
    }
    if constexpr (!G::TRACKED) {
        ring_wait<(R - 1) * G::LPS>();
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int f = 0; f < G::NFR; ++f) ring_ready(ring.r[ST % R][k][f]);
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        const int jn = ST * KS + k + 1;           // the next k-step within the iteration
        const int tap = tap0 + jn / KC, kc = jn % KC;   // and its tap
        if (kc == 0) launder(lane);
        int nb_off[PT];
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) nb_off[pt] = tap_offset<F, PTN, P>(tap_base<F, PTN, P>(tap, pt, lane, bd), kc);
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int t = bb * PT + pt;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    const bf16x8 w_hi = ring.r[ST % R][k][ct * WP];
                    if constexpr (P2 == 2) {
                        mfma_split3(acc[ct][t], w_hi, b[t][0], b[t][1], ring.r[ST % R][k][ct * WP + 1]);
                    } else {
                        acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[t][0], acc[ct][t], 0, 0, 0);
                        if constexpr (P == 2 && PASS == 0) {   // + lo*hi (pass 1: hi*lo only)
                            const bf16x8 w_lo = ring.r[ST % R][k][ct * WP + 1];
                            acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[t][0], acc[ct][t], 0, 0, 0);
                        }
                    }
                }
                {   // tile t of the next k-step (unconditional: past the conv's last k-step the tap
                    // index is 9, whose mask bit is clear, so the reads hit the zero area)
                    const char* a = X + nb_off[pt] + bb * G::ACT_BYTES;
#pragma unroll
                    for (int h = 0; h < P2; ++h) b[t][h] = *(const bf16x8*)(a + h * G::HALF);
                }
                if constexpr (P2 == 1) {   // (the asm chains are not MFMAs to the scheduler)
                    __builtin_amdgcn_sched_group_barrier(0x008, CT * (P == 2 && PASS == 0 ? 2 : 1), 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, P2, 0);                                 // DS read
                }
                if constexpr (EPI && ST == G::U - 1) {
                    if (k == KS - 1 && t >= 1) {
                        if constexpr (P2 == 2) tile_leave(acc, t - 1);
                        epi(t - 1);
                    }
                }
            }
        if constexpr (EPI && ST == G::U - 1) {
            if (k == KS - 1) {
                if constexpr (P2 == 2) tile_leave(acc, G::TT - 1);
                epi(G::TT - 1);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int F, int PTN, int NB, int P, int WG, int PASS, bool EPI, class Epi, int... ST>
__device__ __forceinline__ void conv_iter(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                          f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                          bf16x8 (&b)[Geo<F, PTN, NB, P, WG>::TT][Geo<F, PTN, NB, P, WG>::P2],
                                          const __bf16* wres, uint32_t woff, int gs_it, int gmax, int& lane,
                                          const Board& bd, int tap0, bool last_it, const Epi& epi,
                                          std::integer_sequence<int, ST...>) {
    (conv_stage_l<F, PTN, NB, P, WG, PASS, ST, EPI, Epi>(X, ring, acc, b, wres, woff, gs_it, gmax, lane, bd, tap0, last_it,
                                                         epi), ...);
}

// PASS (P = 2): 0 starts the accumulators, 1 adds to them.  EPI: the epilogue epi(t) of every
// position tile runs inside the last iteration (conv_stage_l), the last iteration peeled.
template <int F, int PTN, int NB, int P, int WG = 1, int PASS = 0, bool EPI = false, class Epi = NoEpi>
__device__ __forceinline__ void conv3x3_looped(const char* __restrict__ X, Ring<F, PTN, NB, P, WG>& ring,
                                               f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                               const __bf16* wres, uint32_t woff, int gs0, int gmax, int lane,
                                               const Board& bd, const Epi& epi = Epi{}) {
    using G = Geo<F, PTN, NB, P, WG>;
    constexpr int PT = G::PT, TT = G::TT;
    if constexpr (PASS == 0) {
#pragma unroll
        for (int ct = 0; ct < G::CT; ++ct)
#pragma unroll
            for (int t = 0; t < TT; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    bf16x8 b[TT][G::P2];
    launder(lane);
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
        const char* a = X + tap_offset<F, PTN, P>(tap_base<F, PTN, P>(0, pt, lane, bd), 0);
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
#pragma unroll
            for (int h = 0; h < G::P2; ++h) b[bb * PT + pt][h] = *(const bf16x8*)(a + bb * G::ACT_BYTES + h * G::HALF);
    }
    if constexpr (G::P2 == 2) split_chain_enter(acc);
    constexpr int NLOOP = EPI ? G::NIT - 1 : G::NIT;
#pragma clang loop unroll(disable)
    for (int it = 0; it < NLOOP; ++it)
        conv_iter<F, PTN, NB, P, WG, PASS, false, NoEpi>(X, ring, acc, b, wres, woff, gs0 + it * G::U, gmax, lane, bd,
                                                       it * G::TPI, it == G::NIT - 1, NoEpi{},
                                                       std::make_integer_sequence<int, G::U>{});
    if constexpr (EPI)
        conv_iter<F, PTN, NB, P, WG, PASS, true, Epi>(X, ring, acc, b, wres, woff, gs0 + NLOOP * G::U, gmax, lane, bd,
                                                   NLOOP * G::TPI, true, epi, std::make_integer_sequence<int, G::U>{});
    if constexpr (G::P2 == 2) split_chain_leave(acc);
}

// Per-board channel sums over the board's positions of the wave's accumulator tiles: lane group g
// (lanes 16g .. 16g+15) ends with the sums of channels co_base + 16ct + 4g + r in every lane.  The
// order (tiles ascending, then a butterfly over the 16 lanes) depends only on the board.
template <int F, int PTN, int NB, int P, int WG = 1>
__device__ __forceinline__ f32x4 board_channel_sum(const f32x4 (&acc)[Geo<F, PTN, NB, P, WG>::CT][Geo<F, PTN, NB, P, WG>::TT],
                                                   int ct, int bb, int li, int npos) {
    using G = Geo<F, PTN, NB, P, WG>;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pt = 0; pt < G::PT; ++pt)
        if (16 * pt + li < npos) {
            const f32x4 v = acc[ct][bb * G::PT + pt];
            s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
        }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] += __shfl_xor(s[r], o, 64);
    return s;
}

// Squeeze-excite gate of v2 block `blk` (model.py:101-126) applied in place to the conv2 output in
// acc: per board, channel means -> Dense(S) relu -> Dense(F) sigmoid -> scale.  Two workgroup
// barriers (every wave must reach this).  ses = LDS scratch of se_scratch_bytes(F, NB).
template <int F, int PTN, int NB, int P>
__device__ __forceinline__ void squeeze_excite(const KParams& kp,
                                               f32x4 (&acc)[Geo<F, PTN, NB, P>::CT][Geo<F, PTN, NB, P>::TT], int blk,
                                               float* ses, int co_base, int lane) {
    using G = Geo<F, PTN, NB, P>;
    constexpr int CT = G::CT, PT = G::PT;
    const int g = lane >> 4, li = lane & 15, npos = kp.npos, S = kp.S;
    float* mean = ses;                 // [NB][F]
    float* hid = ses + NB * F;         // [NB][kMaxSE]
    const float inv = 1.f / (float)npos;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const f32x4 s = board_channel_sum<F, PTN, NB, P>(acc, ct, bb, li, npos);
            if (li == 0)
                *(float4*)(mean + bb * F + co_base + 16 * ct + 4 * g) =
                    make_float4(s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv);
        }
    __syncthreads();
    const float* w1 = kp.sew1 + (size_t)blk * F * S;
    for (int i = threadIdx.x; i < NB * S; i += 256) {
        const int bb = i / S, j = i - bb * S;
        float h = 0.f;
        for (int c = 0; c < F; ++c) h += mean[bb * F + c] * w1[c * S + j];
        hid[bb * kMaxSE + j] = fmaxf(h, 0.f);
    }
    __syncthreads();
    const float* w2 = kp.sew2 + (size_t)blk * S * F;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int co = co_base + 16 * ct + 4 * g;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            float z0 = 0.f, z1 = 0.f, z2 = 0.f, z3 = 0.f;
            for (int j = 0; j < S; ++j) {
                const float h = hid[bb * kMaxSE + j];
                const float4 w = *(const float4*)(w2 + (size_t)j * F + co);
                z0 += h * w.x; z1 += h * w.y; z2 += h * w.z; z3 += h * w.w;
            }
            const float g0 = 1.f / (1.f + __expf(-z0)), g1 = 1.f / (1.f + __expf(-z1));
            const float g2 = 1.f / (1.f + __expf(-z2)), g3 = 1.f / (1.f + __expf(-z3));
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                f32x4& v = acc[ct][bb * PT + pt];
                v[0] *= g0; v[1] *= g1; v[2] *= g2; v[3] *= g3;
            }
        }
    }
}

// v2 pre-activation of the stream for block blk's first conv: act(s * scale + shift)
__device__ __forceinline__ f32x4 pre_act(f32x4 v, const float4& sc, const float4& sh, int leaky) {
    v[0] = act_fn(v[0] * sc.x + sh.x, leaky);
    v[1] = act_fn(v[1] * sc.y + sh.y, leaky);
    v[2] = act_fn(v[2] * sc.z + sh.z, leaky);
    v[3] = act_fn(v[3] * sc.w + sh.w, leaky);
    return v;
}

// P = 2, after an epilogue wrote the lo parts of the image (and a barrier): copy them to the
// workgroup's lo scratch in device memory, then write the hi parts of acc into the image.
// LD = true: the other direction (the lo scratch into the image, for a conv's second pass).
template <int F, int PTN, bool LD>
__device__ __forceinline__ void lo_copy(char* X, char* xlo, int npos, int tid) {
    using G = Geo<F, PTN, 1, 2>;
    const int n16 = npos * G::ROWS / 16;   // the on-board rows (the zero and scratch rows stay)
    uint4* img = (uint4*)X;
    uint4* glo = (uint4*)xlo;
    if constexpr (LD) {
        // LDS-DMA (global_load_lds_dwordx4): each wave-instruction moves 64 consecutive uint4 (1 KB)
        // from the scratch straight into the image -- no VGPR staging, so every load of the thread is
        // in flight at once instead of 4 per round trip (the copy was 12 % of cfg4's kernel time)
        const int lane = tid & 63;
        for (int i0 = tid - lane; i0 < n16; i0 += 256) {
            if (i0 + lane < n16)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(glo + i0 + lane),
                                                 (__attribute__((address_space(3))) void*)(img + i0), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll 4
        for (int i = tid; i < n16; i += 256) glo[i] = img[i];
    }
}
template <int F, int PTN>
__device__ __forceinline__ void save_lo_write_hi(char* X, char* xlo, const f32x4 (&acc)[Geo<F, PTN, 1, 2>::CT][Geo<F, PTN, 1, 2>::TT],
                                                 int npos, int tid, int co_base, int li, int g) {
    using G = Geo<F, PTN, 1, 2>;
    lo_copy<F, PTN, false>(X, xlo, npos, tid);
    // the image may be overwritten once every wave's LDS reads of it are done; the scratch stores
    // drain in the background (the next workgroup barrier with a fence, at the end of the next conv's
    // first pass, orders them before the copy back)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int ct = 0; ct < G::CT; ++ct)
#pragma unroll
        for (int t = 0; t < G::TT; ++t) store_act<F, PTN, 1, false>(X, 16 * t + li, co_base + 16 * ct + 4 * g, acc[ct][t], npos);
    __syncthreads();
}

// The trunk of NB boards per workgroup of 4 waves (trunk_kernel / trunk_kernel_v2 below).  V2:
// pre-activation blocks with optional squeeze-excite (a separate instantiation, so the v1 kernels'
// register allocation is not burdened by the v2 epilogues).
template <int F, int PTN, int NB, int WPE, int P, bool V2, int WG = 1>
__device__ __forceinline__ void trunk_body(const KParams& kp) {
    using G = Geo<F, PTN, NB, P, WG>;
    static_assert(P == 1 || (P == 3 && (NB == 1 || G::WRAP) && (G::CT * G::TT <= 16 || G::SI)) || (P == 2 && G::SI && (!V2 || kLoDirect)),
                  "split precision: F <= 128 (F = 256: single image)");
    constexpr int P2 = G::P2;
    constexpr int IP2 = G::WP;    // bf16 parts of the initial conv's operands (im2col scratch, w0 / w0lo)
    constexpr int PT = G::PT, TT = G::TT, CT = G::CT, R = G::R, NWV = G::NWV, NGR = G::NGR, kThreads = 64 * NWV;
    const int NPOS = kp.npos, H = kp.H, W = kp.W;     // the board (NPOS <= G::NPOS)
    Board bd{H, W, NPOS, kp.wmagic, {}};
    {
        const int li = threadIdx.x & 15;
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
            const int p = 16 * pt + li;
            const int r = bd.row(p), x = p - r * W;
            int m = 0;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int y = r + tap / 3 - 1, xx = x + tap % 3 - 1;
                if (p < NPOS && (unsigned)y < (unsigned)H && (unsigned)xx < (unsigned)W) m |= 1 << tap;
            }
            bd.tapmask[pt] = m;
        }
    }
    constexpr int ACT = G::ACT_BYTES;

    constexpr bool SI = G::SI, RG = G::RG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // wave group grp (WG = 2: threads 256 grp .. 256 grp + 255) takes boards NB grp .. of the
    // workgroup; LDS: image set 0 [WG][NB][ACT], image set 1 [WG][NB][ACT], bias table
    const int grp = NGR == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kThreads));
    char* X0 = smem + grp * NB * ACT;                                  // [NB][ACT]
    char* X1 = SI ? smem : smem + NGR * NB * ACT + grp * NB * ACT;      // [NB][ACT]
    char* SCR = X1;                  // scratch aliases X1 while X1 holds no live activations
    char* SCR0 = SI ? smem : smem + NGR * NB * ACT;   // group 0's scratch (the fused heads' shared features)
    float* btab = (float*)(smem + kp.btab_off);   // trunk conv biases [2B][F], after X1 / scratch

    const int board0 = (blockIdx.x * NGR + grp) * NB;
    const int tid = threadIdx.x & (kThreads - 1);   // within the group
#define GZ_STAMP(i) \
    if (kp.stamps && threadIdx.x == 0) kp.stamps[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime()
    GZ_STAMP(0);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int co_base = wave * (F / NWV);
    const int C = kp.C, K0 = kp.K0;

    // The NB boards' input planes, fetched before anything else with 16-byte loads so that one round
    // trip (pinned host memory over PCIe in the runner, HBM otherwise) covers every board: up to
    // kPF float4 per thread per board, when the plane block is a whole number of aligned float4s
    // (otherwise the staging loop below reads it)
    constexpr int kPF = 4;
    const int nf4 = (C * NPOS) >> 2;
    const float* in_b[NB];
    bool vec_b[NB];
    float4 pf[NB][kPF];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const bool live = board0 + bb < kp.n;
        const int sg = find_segment(kp, board0 + bb);
        in_b[bb] = live ? kp.seg[sg].planes + (size_t)(board0 + bb - kp.seg[sg].row0) * C * NPOS : nullptr;
        vec_b[bb] = ((C * NPOS) & 3) == 0 && nf4 <= kPF * kThreads && ((uintptr_t)in_b[bb] & 15) == 0;
#pragma unroll
        for (int k = 0; k < kPF; ++k) {
            const int i4 = tid + k * kThreads;
            pf[bb][k] = (live && vec_b[bb] && i4 < nf4) ? ((const float4*)in_b[bb])[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }

    // prime the weight ring: stages 0 .. R-2 of the trunk stream
    static_assert((F / NWV) % 16 == 0, "a wave's output channels are whole 16-channel weight blocks");
    const uint32_t woff = (uint32_t)((co_base >> 4) * G::WP * 1024 + 16 * lane);   // lane's fragment bytes within a k-step
    const int gmax = (P == 2 ? 4 : 2) * kp.B * G::NST - 1;   // P = 2: two passes per conv
    Ring<F, PTN, NB, P, WG> ring;
    if (kp.B > 0) ring_prime<F, PTN, NB, P, WG>(ring, kp.wres, woff, gmax, std::make_integer_sequence<int, R - 1>{});

    f32x4 acc[CT][TT];
    f32x4 resid[RG ? 1 : CT][RG ? 1 : TT];
    // global residual of this wave: tile (ct, t) at rg[(ct * TT + t) * 64]
    f32x4* rg = RG ? kp.resid + ((size_t)(blockIdx.x * 4 + wave) * CT * TT) * 64 + lane : nullptr;
    // P = 2: this workgroup's lo image, after the grid's residual scratch
    char* xlo = P == 2 ? (char*)kp.resid + (size_t)gridDim.x * G::RESID_BYTES + (size_t)blockIdx.x * G::LO_BYTES : nullptr;

    // concat_all_layers value head (V2 nets, model.py:251-260): trunk layer j's 1x1 value conv from
    // the fp32 stream in acc -- per-wave partial sums of board bb into LDS (cal_partial), summed in a
    // fixed order, biased and activated after the next workgroup barrier (cal_reduce) into the
    // device feature scratch, which heads_kernel reads.  The partials are rewritten only after at
    // least one more barrier (the next block's first epilogue), so one buffer serves every layer.
    float* calp = (float*)(smem + kp.cal_off);   // [4 waves][NB][NPOS]
    // (gz_nn.hip sizes cal_off's buffer and cal_reduce sums for exactly four waves)
    static_assert(!V2 || NWV == 4, "concat_all_layers partials: four waves per group");
    auto cal_partial = [&](int j, int bb) {
        float4 wv[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) wv[ct] = *(const float4*)(kp.wcl + (size_t)j * F + co_base + 16 * ct + 4 * g);
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
            float sum = 0.f;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const f32x4 a = acc[ct][bb * PT + pt];
                sum += a[0] * wv[ct].x;
                sum += a[1] * wv[ct].y;
                sum += a[2] * wv[ct].z;
                sum += a[3] * wv[ct].w;
            }
            sum += __shfl_xor(sum, 16, 64);
            sum += __shfl_xor(sum, 32, 64);
            const int p = 16 * pt + li;
            if (g == 0 && p < NPOS) calp[(wave * NB + bb) * NPOS + p] = sum;
        }
    };
    auto cal_reduce = [&](int j) {
        for (int i = tid; i < NB * NPOS; i += kThreads) {
            const int bb = i / NPOS, p = i - bb * NPOS;
            const int board = board0 + bb;
            if (board >= kp.n) continue;
            float sum = kp.bcl[j];
#pragma unroll
            for (int w = 0; w < 4; ++w) sum += calp[(w * NB + bb) * NPOS + p];
            kp.feat[(size_t)board * kp.FS + 2 * kp.R * NPOS + j * NPOS + p] = act_fn(sum, kp.leaky);
        }
    };

    for (int i = threadIdx.x; i < 2 * kp.B * F; i += kThreads * NGR) btab[i] = kp.bres[i];
    for (int i = tid; i < NB * G::ZROWS * G::ROWS / 4; i += kThreads) {
        const int bb = i / (G::ZROWS * G::ROWS / 4), j = i % (G::ZROWS * G::ROWS / 4);
        ((uint32_t*)(X0 + bb * ACT + NPOS * G::ROWS))[j] = 0u;
    }

    // ---- per board: stage planes, im2col, initial conv (GEMM over K0) ----------------------
    float* sin = (float*)SCR;
    char* IM = SCR + align16(C * NPOS * 4);
    const int imrow = K0 * 2;
    char* IMlo = IM + align16((NPOS + 1) * imrow);   // split precision: lo parts of the inputs
    // chunk swizzle of an im2col row: XOR with (p & imswz) must map the row's K0 / 8 chunks onto
    // themselves, so imswz + 1 is the largest power of two (<= 16) dividing the chunk count (K0 = 32,
    // 64, 128: 3, 7, 15).  (Rounds 1-4 took min(chunks, 16) - 1, which for K0 = 96 / 160 / 224 -- a
    // 3x3 initial conv over 8-10 / 15-17 / 22-24 planes -- sent chunks past the row into the next
    // position's: the draughts model file f1_581 computed wrong inputs, hidden in bf16's tolerance.)
    const int nch0 = K0 >> 3;
    const int imswz = ((nch0 & -nch0) < 16 ? (nch0 & -nch0) : 16) - 1;
    // initial-conv weights one k-step ahead of their MFMAs (each step's fragments would otherwise
    // wait a full L2 round trip); the first step's are the same for every board: issued here, with
    // the input planes still in flight
    const int nk0 = K0 >> 5;
    auto load_w0 = [&](int s, bf16x8 (&x)[CT], bf16x8 (&xl)[CT]) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const size_t o = ((size_t)(s * F + co_base + 16 * ct + li)) * 32 + 8 * g;
            x[ct] = *(const bf16x8*)(kp.w0 + o);
            if constexpr (IP2 == 2) xl[ct] = *(const bf16x8*)(kp.w0lo + o);
        }
    };
    bf16x8 a0[CT], alo0[CT];
    load_w0(0, a0, alo0);
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const float* in = in_b[bb];
        if (vec_b[bb]) {   // dead boards: zeros
#pragma unroll
            for (int k = 0; k < kPF; ++k)
                if (tid + k * kThreads < nf4) ((float4*)sin)[tid + k * kThreads] = pf[bb][k];
        } else {
            for (int i = tid; i < C * NPOS; i += kThreads) sin[i] = in != nullptr ? in[i] : 0.f;
        }
        // IM[p][k], k = tap*C + c (a 1x1 initial conv: k = c), zero padded to K0: zero the image
        // (beside the planes' staging: disjoint; once per workgroup where the image survives the
        // board -- the entries the copy below writes depend on the geometry only), then one thread
        // per (position, tap) copies its C channels (compile-time divisors only)
        if (SI || bb == 0)
            for (int i = tid; i < IP2 * align16((NPOS + 1) * imrow) / 16; i += kThreads) ((uint4*)IM)[i] = uint4{0u, 0u, 0u, 0u};
        __syncthreads();
        const int T0 = kp.k0taps;
        for (int i = tid; i < NPOS * T0; i += kThreads) {
            int p = i, tap = 4;                // 1x1: the centre tap only
            if (T0 == 9) { p = i / 9; tap = i - p * 9; }
            const int r = bd.row(p);
            const int y = r + tap / 3 - 1, x = p - r * W + tap % 3 - 1;
            if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
                const float* src = sin + y * W + x;
                const int k0 = T0 == 9 ? tap * C : 0;
                for (int c = 0; c < C; ++c) {
                    const int k = k0 + c;
                    const int o = p * imrow + ((((k >> 3) ^ (p & imswz))) << 4) + (k & 7) * 2;
                    const float v = src[c * NPOS];
                    *(__bf16*)(IM + o) = (__bf16)v;
                    if constexpr (IP2 == 2) *(__bf16*)(IMlo + o) = (__bf16)bf16_lo(v);
                }
            }
        }
        __syncthreads();

#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) acc[ct][bb * PT + pt] = f32x4{0.f, 0.f, 0.f, 0.f};
        bf16x8 a[CT], alo[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            a[ct] = a0[ct];
            alo[ct] = alo0[ct];
        }
        for (int s = 0; s < nk0; ++s) {
            bf16x8 an[CT], alon[CT];
            if (s + 1 < nk0) load_w0(s + 1, an, alon);
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int p = 16 * pt + li;
                const int q = p < NPOS ? p : NPOS;
                const int o = q * imrow + ((((s * 4 + g)) ^ (q & imswz)) << 4);
                const bf16x8 bq = *(const bf16x8*)(IM + o);
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    f32x4& c = acc[ct][bb * PT + pt];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct], bq, c, 0, 0, 0);
                    if constexpr (IP2 == 2) {
                        const bf16x8 bql = *(const bf16x8*)(IMlo + o);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct], bql, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo[ct], bq, c, 0, 0, 0);
                    }
                }
            }
            if (s + 1 < nk0) {
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    a[ct] = an[ct];
                    if constexpr (IP2 == 2) alo[ct] = alon[ct];
                }
            }
        }
        if constexpr (SI) __syncthreads();    // the image overwrites the im2col scratch
        // v2: the image feeding block 0 is the pre-activation act(BN_1(s)) of the stream
        const bool preact = V2 && kp.B > 0;
        f32x4* rg0 = rg;    // (residual tile addresses formed here, as in the tower's epilogues)
        if constexpr (RG) launder_ptr(rg0);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(kp.b0 + co);
            float4 psc = make_float4(1.f, 1.f, 1.f, 1.f), psh = make_float4(0.f, 0.f, 0.f, 0.f);
            if (preact) {
                psc = *(const float4*)(kp.pre + co);
                psh = *(const float4*)(kp.pre + F + co);
            }
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                f32x4 v = acc[ct][bb * PT + pt];
                v[0] += bias.x; v[1] += bias.y; v[2] += bias.z; v[3] += bias.w;
                if (!V2 || kp.init_act) {
                    v[0] = act_fn(v[0], kp.leaky);
                    v[1] = act_fn(v[1], kp.leaky);
                    v[2] = act_fn(v[2], kp.leaky);
                    v[3] = act_fn(v[3], kp.leaky);
                }
                if constexpr (RG) rg0[(ct * TT + bb * PT + pt) * 64] = v;
                else resid[ct][bb * PT + pt] = v;
                acc[ct][bb * PT + pt] = v;    // the heads read acc when there is no residual block
                if constexpr (P == 2 && kLoDirect) {
                    const f32x4 sv = preact ? pre_act(v, psc, psh, kp.leaky) : v;
                    store_act<F, PTN, 1, false>(X0 + bb * ACT, 16 * pt + li, co, sv, NPOS);
                    store_lo_scratch<F, PTN>(xlo, 16 * pt + li, co, sv, NPOS);
                } else {
                    store_act<F, PTN, P, !G::SI>(X0 + bb * ACT, 16 * pt + li, co, preact ? pre_act(v, psc, psh, kp.leaky) : v, NPOS);
                }
            }
        }
        if constexpr (V2)
            if (kp.cal) cal_partial(0, bb);   // layer 0: the initial conv block's output
        __syncthreads();    // scratch is reused by the next board
        if constexpr (P == 2 && !kLoDirect) save_lo_write_hi<F, PTN>(X0, xlo, acc, NPOS, tid, co_base, li, g);
    }
    for (int i = tid; i < NB * G::ZROWS * G::ROWS / 4; i += kThreads) {
        const int bb = i / (G::ZROWS * G::ROWS / 4), j = i % (G::ZROWS * G::ROWS / 4);
        ((uint32_t*)(X1 + bb * ACT + NPOS * G::ROWS))[j] = 0u;
    }
    __syncthreads();
    if constexpr (V2)
        if (kp.cal) cal_reduce(0);

    GZ_STAMP(1);
    // ---- residual tower ------------------------------------------------------------------
    if constexpr (SI) {
        // one image, one conv call site (keeps the fully unrolled F = 256 conv once in the binary)
        for (int cv = 0; cv < 2 * kp.B; ++cv) {
            const bool second = cv & 1;
            const float* bt = btab + cv * F;
            if constexpr (P == 2) {
                if constexpr (G::LOOPSI) conv3x3_looped<F, PTN, NB, P, WG, 0>(X0, ring, acc, kp.wres, woff, (2 * cv) * G::NST, gmax, lane, bd);
                else conv3x3<F, PTN, NB, P, WG, 0>(X0, ring, acc, kp.wres, woff, (2 * cv) * G::NST, gmax, lane, bd);
                __syncthreads();    // every wave has finished reading the hi image
                lo_copy<F, PTN, true>(X0, xlo, NPOS, tid);   // the lo image
                __syncthreads();
                if constexpr (G::LOOPSI) conv3x3_looped<F, PTN, NB, P, WG, 1>(X0, ring, acc, kp.wres, woff, (2 * cv + 1) * G::NST, gmax, lane, bd);
                else conv3x3<F, PTN, NB, P, WG, 1>(X0, ring, acc, kp.wres, woff, (2 * cv + 1) * G::NST, gmax, lane, bd);
            } else if constexpr (G::LOOPSI) {
                conv3x3_looped<F, PTN, NB, P, WG>(X0, ring, acc, kp.wres, woff, cv * G::NST, gmax, lane, bd);
            } else {
                conv3x3<F, PTN, NB, P, WG>(X0, ring, acc, kp.wres, woff, cv * G::NST, gmax, lane, bd);
            }
            __syncthreads();    // every wave has finished reading the image it is about to overwrite
            // residual tile addresses are formed here, not hoisted out of the loop (44 x 64-bit);
            // so are the image's (44 store addresses kept live across the conv spilled)
            f32x4* rgc = rg;
            if constexpr (RG) launder_ptr(rgc);
            char* Xe = X0;
            launder_ptr(Xe);
            char* xloe = xlo;
            if constexpr (P == 2) launder_ptr(xloe);
            int lie = li, ge = g;    // (and their offsets: the lane's row and channel terms)
            launder(lie);
            launder(ge);
            if (V2 && second) {   // v2: s += SE(conv2 + bias); image = act(BN_1 of the next block (s))
                const int blk = cv >> 1;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    const float4 bias = *(const float4*)(bt + co_base + 16 * ct + 4 * g);
#pragma unroll
                    for (int t = 0; t < TT; ++t) {
                        acc[ct][t][0] += bias.x; acc[ct][t][1] += bias.y; acc[ct][t][2] += bias.z; acc[ct][t][3] += bias.w;
                    }
                }
                if (kp.S) squeeze_excite<F, PTN, NB, P>(kp, acc, blk, (float*)(smem + kp.se_off), co_base, lane);
                const bool more = blk + 1 < kp.B;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    const int co = co_base + 16 * ct + 4 * g;
                    float4 psc = make_float4(1.f, 1.f, 1.f, 1.f), psh = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (more) {
                        psc = *(const float4*)(kp.pre + (size_t)(2 * blk + 2) * F + co);
                        psh = *(const float4*)(kp.pre + (size_t)(2 * blk + 3) * F + co);
                    }
#pragma unroll
                    for (int t = 0; t < TT; ++t) {
                        f32x4 v = acc[ct][t], r;
                        if constexpr (RG) r = rgc[(ct * TT + t) * 64];
                        else r = resid[ct][t];
                        v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
                        if constexpr (RG) rgc[(ct * TT + t) * 64] = v;
                        else resid[ct][t] = v;
                        acc[ct][t] = v;
                        if (more) {
                            const f32x4 pv = pre_act(v, psc, psh, kp.leaky);
                            if constexpr (P == 2) {   // (two-pass split: hi parts to the image, lo to the scratch)
                                store_act<F, PTN, 1, false>(Xe, 16 * t + lie, co, pv, NPOS);
                                store_lo_scratch<F, PTN>(xloe, 16 * t + lie, co, pv, NPOS);
                            } else {
                                store_act<F, PTN, P, !G::SI>(X0, 16 * t + li, co, pv, NPOS);
                            }
                        }
                    }
                }
                if (kp.cal)   // layer blk + 1: the block's add
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) cal_partial(blk + 1, bb);
                __syncthreads();
                if (kp.cal) cal_reduce(blk + 1);
                continue;
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const int co = co_base + 16 * ct + 4 * ge;
                const float4 bias = *(const float4*)(bt + co);
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    f32x4 v = acc[ct][t];
                    v[0] += bias.x; v[1] += bias.y; v[2] += bias.z; v[3] += bias.w;
                    if (second) {
                        f32x4 r;
                        if constexpr (RG) r = rgc[(ct * TT + t) * 64];
                        else r = resid[ct][t];
                        v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
                    }
                    v[0] = act_fn(v[0], kp.leaky);
                    v[1] = act_fn(v[1], kp.leaky);
                    v[2] = act_fn(v[2], kp.leaky);
                    v[3] = act_fn(v[3], kp.leaky);
                    if (second) {
                        if constexpr (RG) rgc[(ct * TT + t) * 64] = v;
                        else resid[ct][t] = v;
                    }
                    if constexpr (P == 2 && kLoDirect) {
                        if (second) acc[ct][t] = v;
                        store_act<F, PTN, 1, false>(Xe, 16 * t + lie, co, v, NPOS);
                        store_lo_scratch<F, PTN>(xloe, 16 * t + lie, co, v, NPOS);
                    } else {
                        if (second || P == 2) acc[ct][t] = v;
                        store_act<F, PTN, P, !G::SI>(Xe, 16 * t + lie, co, v, NPOS);
                    }
                }
            }
            __syncthreads();
            if constexpr (P == 2 && !kLoDirect) save_lo_write_hi<F, PTN>(Xe, xlo, acc, NPOS, tid, co_base, lie, ge);
        }
    } else
    for (int blk = 0; blk < kp.B; ++blk) {
        const float alpha = kp.leaky ? 0.03f : 0.f;
        const float* b_a = btab + (2 * blk) * F;
        const float* b_b = b_a + F;

        if constexpr (!V2 && G::LOOP && kEpiInConv) {
            // the same two epilogues as below, run per position tile inside each conv's last k-step
            float4 bia[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) bia[ct] = *(const float4*)(b_a + co_base + 16 * ct + 4 * g);
            auto epi1 = [&](int t) {
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    f32x4 v = acc[ct][t];
                    v[0] = act_mx(v[0] + bia[ct].x, alpha);
                    v[1] = act_mx(v[1] + bia[ct].y, alpha);
                    v[2] = act_mx(v[2] + bia[ct].z, alpha);
                    v[3] = act_mx(v[3] + bia[ct].w, alpha);
                    store_act<F, PTN, P, !G::SI>(X1 + (t / PT) * ACT, 16 * (t % PT) + li, co_base + 16 * ct + 4 * g, v, NPOS);
                }
            };
            conv3x3_looped<F, PTN, NB, P, WG, 0, true>(X0, ring, acc, kp.wres, woff, (2 * blk) * G::NST, gmax, lane, bd, epi1);
            __syncthreads();
            float4 bib[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) bib[ct] = *(const float4*)(b_b + co_base + 16 * ct + 4 * g);
            auto epi2 = [&](int t) {
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    f32x4 v = acc[ct][t];
                    const f32x4 r = resid[ct][t];
                    v[0] = act_mx(v[0] + bib[ct].x + r[0], alpha);
                    v[1] = act_mx(v[1] + bib[ct].y + r[1], alpha);
                    v[2] = act_mx(v[2] + bib[ct].z + r[2], alpha);
                    v[3] = act_mx(v[3] + bib[ct].w + r[3], alpha);
                    resid[ct][t] = v;
                    acc[ct][t] = v;
                    store_act<F, PTN, P, !G::SI>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co_base + 16 * ct + 4 * g, v, NPOS);
                }
            };
            conv3x3_looped<F, PTN, NB, P, WG, 0, true>(X1, ring, acc, kp.wres, woff, (2 * blk + 1) * G::NST, gmax, lane, bd, epi2);
            __syncthreads();
            continue;
        }
        if constexpr (G::LOOP) conv3x3_looped<F, PTN, NB, P, WG>(X0, ring, acc, kp.wres, woff, (2 * blk) * G::NST, gmax, lane, bd);
        else conv3x3<F, PTN, NB, P, WG>(X0, ring, acc, kp.wres, woff, (2 * blk) * G::NST, gmax, lane, bd);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(b_a + co);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 v = acc[ct][t];
                v[0] = act_mx(v[0] + bias.x, alpha);
                v[1] = act_mx(v[1] + bias.y, alpha);
                v[2] = act_mx(v[2] + bias.z, alpha);
                v[3] = act_mx(v[3] + bias.w, alpha);
                store_act<F, PTN, P, !G::SI>(X1 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);
            }
        }
        __syncthreads();

        if constexpr (G::LOOP) conv3x3_looped<F, PTN, NB, P, WG>(X1, ring, acc, kp.wres, woff, (2 * blk + 1) * G::NST, gmax, lane, bd);
        else conv3x3<F, PTN, NB, P, WG>(X1, ring, acc, kp.wres, woff, (2 * blk + 1) * G::NST, gmax, lane, bd);
        if constexpr (V2) {   // s += SE(conv2 + bias); image = act(BN_1 of the next block (s)), model.py:128-149
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const float4 bias = *(const float4*)(b_b + co_base + 16 * ct + 4 * g);
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    acc[ct][t][0] += bias.x; acc[ct][t][1] += bias.y; acc[ct][t][2] += bias.z; acc[ct][t][3] += bias.w;
                }
            }
            if (kp.S) squeeze_excite<F, PTN, NB, P>(kp, acc, blk, (float*)(smem + kp.se_off), co_base, lane);
            const bool more = blk + 1 < kp.B;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const int co = co_base + 16 * ct + 4 * g;
                float4 psc = make_float4(1.f, 1.f, 1.f, 1.f), psh = make_float4(0.f, 0.f, 0.f, 0.f);
                if (more) {
                    psc = *(const float4*)(kp.pre + (size_t)(2 * blk + 2) * F + co);
                    psh = *(const float4*)(kp.pre + (size_t)(2 * blk + 3) * F + co);
                }
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    f32x4 v = acc[ct][t];
                    const f32x4 r = resid[ct][t];
                    v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
                    resid[ct][t] = v;
                    acc[ct][t] = v;
                    if (more) store_act<F, PTN, P, !G::SI>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co, pre_act(v, psc, psh, kp.leaky), NPOS);
                }
            }
            if (kp.cal)   // layer blk + 1: the block's add
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) cal_partial(blk + 1, bb);
            __syncthreads();
            if (kp.cal) cal_reduce(blk + 1);
            continue;
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int co = co_base + 16 * ct + 4 * g;
            const float4 bias = *(const float4*)(b_b + co);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 v = acc[ct][t];
                const f32x4 r = resid[ct][t];
                v[0] = act_mx(v[0] + bias.x + r[0], alpha);
                v[1] = act_mx(v[1] + bias.y + r[1], alpha);
                v[2] = act_mx(v[2] + bias.z + r[2], alpha);
                v[3] = act_mx(v[3] + bias.w + r[3], alpha);
                resid[ct][t] = v;
                acc[ct][t] = v;
                store_act<F, PTN, P, !G::SI>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);
            }
        }
        __syncthreads();
    }
    // the clamped tail stages are never consumed: land them before their registers are released
    if (!G::TRACKED && kp.B > 0) {
        ring_wait<0>();
#pragma unroll
        for (int s = 0; s < R; ++s)
#pragma unroll
            for (int k = 0; k < G::KS; ++k)
#pragma unroll
                for (int f = 0; f < G::NFR; ++f) ring_ready(ring.r[s][k][f]);
    }

    GZ_STAMP(2);
    // ---- the heads' 1x1 convs (2 per policy role + 1 value) from the fp32 residual stream (a copy
    // of the last epilogue's output is in acc);
    // features in the model's Flatten order go to the scratch for heads_kernel ----------------
    const int HC = 2 * kp.R + (kp.cal ? 0 : 1);   // (concat_all_layers: the value features are written)
    // head-conv partials per 16-channel tile (the same sums whatever the waves' channel split, so
    // every variant -- 4 or 8 waves -- computes every row identically)
    constexpr int NT16 = F / 16;
    float* hpart = (float*)SCR;                                  // [NB][NT16][HC][NPOS]
    // the heads' 1x1 conv weights of this wave's channels, loaded together once for the NB boards
    // (two-role games, F <= 128) instead of one dependent global load per conv and board
    constexpr int kHoistHC = 5;
    constexpr bool HOIST_WH = !SI && CT <= 2;
    float4 whv[HOIST_WH ? kHoistHC : 1][CT];
    if constexpr (HOIST_WH) {
        if (HC <= kHoistHC) {
#pragma unroll
            for (int h = 0; h < kHoistHC; ++h)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
                    if (h < HC) whv[h][ct] = *(const float4*)(kp.wh + (size_t)h * F + co_base + 16 * ct + 4 * g);
        }
    }
    // FUSE (two-image kernels): the features stay in LDS, fk = [FS][NB], and the dense heads run
    // here; single-image kernels write them to the device scratch for heads_kernel
    // (WG = 2: each group's 1x1 partials in its own scratch, the features of the workgroup's boards
    // in group 0's, after its partials)
    constexpr bool FUSE = !SI;
    const bool fuse = FUSE && !kp.nofuse;   // nofuse: the features go to the device scratch
    constexpr int NBW = NB * NGR;    // boards per workgroup
    float* fk = (float*)(SCR0 + align16(NB * NT16 * HC * NPOS * 4));
    float* lg = fk + align16(kp.FS * NBW * 4) / 4;
    // feature k of board bb
    auto feat_at = [&](int bb, int k) -> float& {
        if (fuse) return fk[k * NBW + grp * NB + bb];
        return kp.feat[(size_t)(board0 + bb) * kp.FS + k];
    };
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const int board = board0 + bb;
        if (kp.gapF && board < kp.n) {   // pooling value head: the trunk's channel means (model.py:263)
            const float inv = 1.f / (float)NPOS;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const f32x4 sm = board_channel_sum<F, PTN, NB, P, WG>(acc, ct, bb, li, NPOS);
                const int co = co_base + 16 * ct + 4 * g;
                if (li == 0)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (co + r < kp.gapF) feat_at(bb, 2 * kp.R * NPOS + co + r) = sm[r] * inv;
            }
        }
        // one 1x1 head conv (output h) of board bb from the fp32 stream, weights wv
        auto head_conv = [&](int h, const float4 (&wv)[CT]) {
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) {
                const int p = 16 * pt + li;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    const f32x4 a = acc[ct][bb * PT + pt];
                    float s = a[0] * wv[ct].x;
                    s += a[1] * wv[ct].y;
                    s += a[2] * wv[ct].z;
                    s += a[3] * wv[ct].w;
                    s += __shfl_xor(s, 16, 64);
                    s += __shfl_xor(s, 32, 64);
                    if (g == 0 && p < NPOS) hpart[((bb * NT16 + co_base / 16 + ct) * HC + h) * NPOS + p] = s;
                }
            }
        };
        if constexpr (HOIST_WH) {
            if (HC <= kHoistHC) {
#pragma unroll
                for (int h = 0; h < kHoistHC; ++h)
                    if (h < HC) head_conv(h, whv[h]);
            }
        }
        if (!HOIST_WH || HC > kHoistHC) {
            for (int h = 0; h < HC; ++h) {
                float4 wv[CT];
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) wv[ct] = *(const float4*)(kp.wh + (size_t)h * F + co_base + 16 * ct + 4 * g);
                head_conv(h, wv);
            }
        }
    }
    // every board's partials summed in one pass (one barrier pair for the NB boards)
    __syncthreads();
    for (int i = tid; i < NB * HC * NPOS; i += kThreads) {
        const int bb = i / (HC * NPOS), hp = i - bb * (HC * NPOS);
        const int h = hp / NPOS, p = hp - h * NPOS;
        if (board0 + bb >= kp.n) continue;
        float s = kp.bh[h];
#pragma unroll
        for (int w = 0; w < NT16; ++w) s += hpart[((bb * NT16 + w) * HC + h) * NPOS + p];
        s = act_fn(s, kp.leaky);
        if (h < 2 * kp.R) {
            const int r = h >> 1, c = h & 1;
            const int idx = kp.flatten_nchw ? c * NPOS + p : p * 2 + c;
            feat_at(bb, r * 2 * NPOS + idx) = s;
        } else {
            feat_at(bb, 2 * kp.R * NPOS + kp.gapF + p) = s;
        }
    }
    __syncthreads();
    GZ_STAMP(3);
    if (fuse) {
        const int wb0 = blockIdx.x * NBW;
        const int nb = kp.n - wb0 < NBW ? kp.n - wb0 : NBW;
        dense_heads<NBW, kThreads * NGR>(kp, fk, lg, wb0, nb);
    }
    GZ_STAMP(4);
#undef GZ_STAMP
}

// WPE = minimum resident waves per SIMD the register allocation must allow (amdgpu_waves_per_eu),
// i.e. WPE workgroups per CU.
template <int F, int PTN, int NB, int WPE, int P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
trunk_kernel(const KParams kp) {
    trunk_body<F, PTN, NB, WPE, P, false>(kp);
}

// Two wave groups of 4 (8 waves, two per SIMD, a board per group): while one wave waits on a
// barrier, an LDS read or its epilogue, the other wave of its SIMD issues MFMAs.  Same LDS as the
// two-board kernel; each group streams the weights itself (twice the L2 weight traffic).
template <int F, int PTN, int P>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
trunk_kernel8(const KParams kp) {
    trunk_body<F, PTN, 1, 2, P, false, 2>(kp);
}

// One group of 8 waves (two per SIMD) for two boards, each wave half of the 4-wave kernel's output
// channels (variant 24): the weight stream per workgroup stays that of trunk_kernel<.., 2, ..>, the B
// fragments are read by twice as many waves
template <int F, int PTN, int P>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
trunk_kernel_w8(const KParams kp) {
    trunk_body<F, PTN, 2, 2, P, false, 3>(kp);
}

// Two wave groups of 2 (4 waves, one per SIMD, a board per group; variant 23): each wave multiplies
// 4 co tiles by its board's position tiles, so a k-step reads half the B fragments of the two-board
// kernel for the same MFMAs and streams twice the weight fragments
template <int F, int PTN, int P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
trunk_kernel_h2(const KParams kp) {
    trunk_body<F, PTN, 1, 1, P, false, 4>(kp);
}

template <int F, int PTN, int NB, int WPE, int P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
trunk_kernel_v2(const KParams kp) {
    trunk_body<F, PTN, NB, WPE, P, true>(kp);
}

// ---- heads -------------------------------------------------------------------------------------
// Dense heads of BPW boards whose head features are in LDS, fk = [FS][BPW] (k-major, board-minor):
// policy Dense + softmax per role, value MLP + softmax (sigmoid for legacy files); results straight
// to the segments' buffers.  lg = LDS [BPW][LMAX].  Dense layers in fp32: thread j owns output j
// (of P_r or VH) for every board; the k-major weights are read coalesced, once per call, and the
// features come from LDS as one broadcast read per k.  Each board's sums run in a fixed k order with
// the same operations for every BPW, so outputs do not depend on how boards are grouped (fused into
// the trunk kernel with BPW = its NB, or in heads_kernel with BPW = 4).  Every thread of the
// workgroup (4 waves) must call it; boards board0 .. board0 + nb - 1 are written.
constexpr int kGemmSoftmaxMax = 3072;   // policy rows the register softmax of gemm_heads takes (48 per lane)

template <int BPW, int NT>
__device__ __forceinline__ void dense_heads_seq(const KParams& kp, const float* fk, float* lg, int board0, int nb) {
    static_assert(BPW >= 1 && BPW <= 4, "one softmax wave per board");
    const int NPOS = kp.npos;
    const int LMAX = kp.lgrow;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // policy heads: Dense(2HW -> P_r) + softmax
    for (int r = 0; r < kp.R; ++r) {
        const int P = kp.P[r], K = 2 * NPOS;
        const float* Wd = kp.pd[r];
        const float* fr = fk + (size_t)r * 2 * NPOS * BPW;
        int lof = 0;
        for (int q = 0; q < r; ++q) lof += kp.P[q];
        if (kp.gemm_heads && P <= kGemmSoftmaxMax) {
            // logits computed by policy_gemm_kernel (bias included): wave b takes board b's row
            // straight from the logits scratch into registers -- every load of the row in flight at
            // once instead of a load / LDS-store round trip per 256 values -- with the same
            // per-lane order (j = lane, lane + 64, ...) and reductions as the LDS path below
            if (wave < nb) {
                constexpr int NV = kGemmSoftmaxMax / 64;
                const int b = wave, board = board0 + b;
                const float* l = kp.glog + (size_t)board * kp.plog + lof;
                float v[NV];
#pragma unroll
                for (int i = 0; i < NV; ++i) v[i] = lane + 64 * i < P ? l[lane + 64 * i] : -3.0e38f;
                float m = -3.0e38f;
#pragma unroll
                for (int i = 0; i < NV; ++i) m = fmaxf(m, v[i]);
                m = wave_max(m);
                float sum = 0.f;
#pragma unroll
                for (int i = 0; i < NV; ++i)
                    if (lane + 64 * i < P) sum += __expf(v[i] - m);
                sum = wave_sum(sum);
                const float inv = 1.f / sum;
                const int sg = find_segment(kp, board);
                float* out = kp.seg[sg].pol[r] + (size_t)(board - kp.seg[sg].row0) * P;
#pragma unroll
                for (int i = 0; i < NV; ++i)
                    if (lane + 64 * i < P) out[lane + 64 * i] = kp.logits ? v[i] : __expf(v[i] - m) * inv;
            }
            continue;
        }
        if (kp.gemm_heads) {   // (rows longer than the register path) through LDS
            for (int i = tid; i < nb * P; i += NT) {
                const int b = i / P, j = i - b * P;
                lg[b * LMAX + j] = kp.glog[(size_t)(board0 + b) * kp.plog + lof + j];
            }
        }
        for (int j = tid; j < P && !kp.gemm_heads; j += NT) {
            float a[BPW];
#pragma unroll
            for (int b = 0; b < BPW; ++b) a[b] = 0.f;
#pragma unroll 32   // many weight loads in flight: the loop is L2-latency bound
            for (int k = 0; k < K; ++k) {
                const float w = Wd[(size_t)k * ((P + 3) & ~3) + j];   // rows padded to P4
#pragma unroll
                for (int b = 0; b < BPW; ++b) a[b] += fr[k * BPW + b] * w;
            }
            const float bj = kp.pb[r][j];
#pragma unroll
            for (int b = 0; b < BPW; ++b) lg[b * LMAX + j] = a[b] + bj;
        }
        __syncthreads();
        if (wave < nb) {                  // wave b: softmax of board b
            const int b = wave;
            const float* l = lg + b * LMAX;
            float m = -3.0e38f;
            for (int j = lane; j < P; j += 64) m = fmaxf(m, l[j]);
            m = wave_max(m);
            float sum = 0.f;
            for (int j = lane; j < P; j += 64) sum += __expf(l[j] - m);
            sum = wave_sum(sum);
            const float inv = 1.f / sum;
            const int board = board0 + b;
            const int sg = find_segment(kp, board);
            float* out = kp.seg[sg].pol[r] + (size_t)(board - kp.seg[sg].row0) * P;
            if (kp.logits) {
                for (int j = lane; j < P; j += 64) out[j] = l[j];
            } else {
                for (int j = lane; j < P; j += 64) out[j] = __expf(l[j] - m) * inv;
            }
        }
        __syncthreads();
    }

    // value head: Dense([GAP F] + HW -> VH) + act, Dense(VH -> V) + softmax
    {
        const int VH = kp.VH, VK = kp.VK;
        const float* fv = fk + (size_t)2 * kp.R * NPOS * BPW;
        for (int j = tid; j < VH; j += NT) {
            float a[BPW];
#pragma unroll
            for (int b = 0; b < BPW; ++b) a[b] = 0.f;
#pragma unroll 32   // many weight loads in flight: the loop is L2-latency bound
            for (int k = 0; k < VK; ++k) {
                const float w = kp.vhw[(size_t)k * ((VH + 3) & ~3) + j];
#pragma unroll
                for (int b = 0; b < BPW; ++b) a[b] += fv[k * BPW + b] * w;
            }
            const float bj = kp.vhb[j];
#pragma unroll
            for (int b = 0; b < BPW; ++b) lg[b * LMAX + j] = act_fn(a[b] + bj, kp.leaky);
        }
        __syncthreads();
        if (wave < nb) {
            const int b = wave;
            const float* hv = lg + b * LMAX;
            float o[4] = {0.f, 0.f, 0.f, 0.f};
            for (int v = 0; v < kp.V; ++v) {
                float sum = 0.f;
                for (int k = lane; k < VH; k += 64) sum += hv[k] * kp.vdw[(size_t)k * kp.V + v];
                o[v] = wave_sum(sum) + kp.vdb[v];
            }
            if (lane == 0) {
                const int board = board0 + b;
                const int sg = find_segment(kp, board);
                float* out = kp.seg[sg].val + (size_t)(board - kp.seg[sg].row0) * kp.V;
                if (kp.logits) {
                    for (int v = 0; v < kp.V; ++v) out[v] = o[v];
                } else if (kp.value_sigmoid) {
                    for (int v = 0; v < kp.V; ++v) out[v] = 1.f / (1.f + __expf(-o[v]));
                } else {
                    float m = o[0];
                    for (int v = 1; v < kp.V; ++v) m = fmaxf(m, o[v]);
                    float e[4], esum = 0.f;
                    for (int v = 0; v < kp.V; ++v) { e[v] = __expf(o[v] - m); esum += e[v]; }
                    for (int v = 0; v < kp.V; ++v) out[v] = e[v] / esum;
                }
            }
        }
    }
}


// Dense heads in two phases (every config whose policy logits are not longer than the register
// softmax takes): (A) every 4-output group of every policy role's Dense and of the value hidden Dense
// is one thread's work, all in flight together -- a thread loads one float4 of 4 consecutive outputs
// per k from the padded [K][N4] weights (gz_nn.hip) and keeps each output's sum in the k order of
// dense_heads_seq, so the results are the same bit for bit -- instead of one Dense after another with
// a barrier and a softmax between them (the weight loads are L2-latency bound); (B) one wave per
// (role, board) softmax and per board's value output.  lg: per board a row of kp.lgrow floats,
// [P4_0 | P4_1 | .. | VH4] (the policy sections absent with gemm_heads).
template <int BPW, int NT>
__device__ __forceinline__ void dense_heads(const KParams& kp, const float* fk, float* lg, int board0, int nb) {
    static_assert(BPW >= 1 && BPW <= 4, "one softmax wave per board");
    if (kp.heads_seq || (kp.gemm_heads && kp.maxP > kGemmSoftmaxMax)) {
        dense_heads_seq<BPW, NT>(kp, fk, lg, board0, nb);
        return;
    }
    const int NPOS = kp.npos, R = kp.R, LG = kp.lgrow;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool gem = kp.gemm_heads != 0;
    int pgroups = 0;
    if (!gem)
        for (int r = 0; r < R; ++r) pgroups += (kp.P[r] + 3) >> 2;
    const int VH4 = (kp.VH + 3) & ~3;
    const int voff = 4 * pgroups;                 // the value section's offset in a board's row
    const int units = pgroups + (VH4 >> 2);
    for (int u = tid; u < units; u += NT) {
        const float* W;
        const float* f;
        int K, N4, q, off, r = 0;
        if (u < pgroups) {
            int uu = u;
            off = 0;
            for (; r < R - 1; ++r) {
                const int g = (kp.P[r] + 3) >> 2;
                if (uu < g) break;
                uu -= g;
                off += 4 * g;
            }
            q = uu;
            W = kp.pd[r];
            N4 = (kp.P[r] + 3) & ~3;
            K = 2 * NPOS;
            f = fk + (size_t)r * 2 * NPOS * BPW;
        } else {
            q = u - pgroups;
            W = kp.vhw;
            N4 = VH4;
            K = kp.VK;
            f = fk + (size_t)2 * R * NPOS * BPW;
            off = voff;
        }
        float a[BPW][4];
#pragma unroll
        for (int b = 0; b < BPW; ++b) a[b][0] = a[b][1] = a[b][2] = a[b][3] = 0.f;
        const float4* w4 = (const float4*)W + q;
        const int rs = N4 >> 2;
#pragma unroll 16   // many weight loads in flight: the loop is L2-latency bound
        for (int k = 0; k < K; ++k) {
            const float4 w = w4[(size_t)k * rs];
#pragma unroll
            for (int b = 0; b < BPW; ++b) {
                const float x = f[k * BPW + b];
                a[b][0] += x * w.x;
                a[b][1] += x * w.y;
                a[b][2] += x * w.z;
                a[b][3] += x * w.w;
            }
        }
        if (u < pgroups) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = 4 * q + i;
                if (j < kp.P[r]) {
                    const float bj = kp.pb[r][j];
#pragma unroll
                    for (int b = 0; b < BPW; ++b) lg[b * LG + off + j] = a[b][i] + bj;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = 4 * q + i;
                if (j < kp.VH) {
                    const float bj = kp.vhb[j];
#pragma unroll
                    for (int b = 0; b < BPW; ++b) lg[b * LG + off + j] = act_fn(a[b][i] + bj, kp.leaky);
                }
            }
        }
    }
    __syncthreads();
    const int ntask = R * nb + nb;
    for (int t = wave; t < ntask; t += NT / 64) {
        if (t < R * nb) {   // softmax of role r, board b
            const int r = t / nb, b = t - r * nb, P = kp.P[r];
            int lof = 0;
            for (int q = 0; q < r; ++q) lof += gem ? kp.P[q] : ((kp.P[q] + 3) & ~3);
            const int board = board0 + b;
            const int sg = find_segment(kp, board);
            float* out = kp.seg[sg].pol[r] + (size_t)(board - kp.seg[sg].row0) * P;
            if (gem) {   // logits from policy_gemm_kernel (bias included), straight into registers
                constexpr int NV = kGemmSoftmaxMax / 64;
                const float* l = kp.glog + (size_t)board * kp.plog + lof;
                float v[NV];
#pragma unroll
                for (int i = 0; i < NV; ++i) v[i] = lane + 64 * i < P ? l[lane + 64 * i] : -3.0e38f;
                float m = -3.0e38f;
#pragma unroll
                for (int i = 0; i < NV; ++i) m = fmaxf(m, v[i]);
                m = wave_max(m);
                float sum = 0.f;
#pragma unroll
                for (int i = 0; i < NV; ++i)
                    if (lane + 64 * i < P) sum += __expf(v[i] - m);
                sum = wave_sum(sum);
                const float inv = 1.f / sum;
#pragma unroll
                for (int i = 0; i < NV; ++i)
                    if (lane + 64 * i < P) out[lane + 64 * i] = kp.logits ? v[i] : __expf(v[i] - m) * inv;
            } else {
                const float* l = lg + b * LG + lof;
                float m = -3.0e38f;
                for (int j = lane; j < P; j += 64) m = fmaxf(m, l[j]);
                m = wave_max(m);
                float sum = 0.f;
                for (int j = lane; j < P; j += 64) sum += __expf(l[j] - m);
                sum = wave_sum(sum);
                const float inv = 1.f / sum;
                if (kp.logits) {
                    for (int j = lane; j < P; j += 64) out[j] = l[j];
                } else {
                    for (int j = lane; j < P; j += 64) out[j] = __expf(l[j] - m) * inv;
                }
            }
        } else {            // value output of board b
            const int b = t - R * nb;
            const float* hv = lg + b * LG + voff;
            float o[4] = {0.f, 0.f, 0.f, 0.f};
            for (int v = 0; v < kp.V; ++v) {
                float sum = 0.f;
                for (int k = lane; k < kp.VH; k += 64) sum += hv[k] * kp.vdw[(size_t)k * kp.V + v];
                o[v] = wave_sum(sum) + kp.vdb[v];
            }
            if (lane == 0) {
                const int board = board0 + b;
                const int sg = find_segment(kp, board);
                float* out = kp.seg[sg].val + (size_t)(board - kp.seg[sg].row0) * kp.V;
                if (kp.logits) {
                    for (int v = 0; v < kp.V; ++v) out[v] = o[v];
                } else if (kp.value_sigmoid) {
                    for (int v = 0; v < kp.V; ++v) out[v] = 1.f / (1.f + __expf(-o[v]));
                } else {
                    float m = o[0];
                    for (int v = 1; v < kp.V; ++v) m = fmaxf(m, o[v]);
                    float e[4], esum = 0.f;
                    for (int v = 0; v < kp.V; ++v) { e[v] = __expf(o[v] - m); esum += e[v]; }
                    for (int v = 0; v < kp.V; ++v) out[v] = e[v] / esum;
                }
            }
        }
    }
}

// floats per board of the dense heads' LDS outputs: the sequential path's max(P, VH) (two = false)
// or the two-phase path's [P4_0 | .. | VH4] row (two = true; at least the former)
__host__ __device__ inline int heads_row(int R, const int* P, int VH, bool two = true) {
    int maxP = 0, sum4 = 0;
    for (int r = 0; r < R; ++r) {
        maxP = P[r] > maxP ? P[r] : maxP;
        sum4 += (P[r] + 3) & ~3;
    }
    const int row = maxP > VH ? maxP : VH;
    const int tw = sum4 + ((VH + 3) & ~3);
    return two && tw > row ? tw : row;
}

// LDS of the fused heads (trunk kernels with two activation images): 1x1-conv partials, features,
// dense outputs (lgrow = heads_row)
// (nb boards per workgroup, nbg of them per wave group; F padded filters: the 1x1-conv partials are
// per group, board and 16-channel tile)
__host__ __device__ inline int fused_heads_bytes(int npos, int R, int lgrow, int gapF, int nb, int nbg, int F) {
    const int FS = (2 * R + 1) * npos + gapF;   // (concat_all_layers nets never fuse the heads)
    return align16(nbg * (F / 16) * (2 * R + 1) * npos * 4) + align16(FS * nb * 4) + align16(nb * lgrow * 4);
}

// Separate heads launch (single-image trunk kernels: kHeadBoards boards per workgroup of features
// from the device scratch).
#ifdef GZNN_DEFINE_HEADS_KERNEL   // defined in one translation unit (gz_nn.hip)
// Policy Dense(2HW -> P_r) of every board of a launch as one GEMM on MFMA (single-image nets with a
// large policy, e.g. amazons P = 3041, where heads_kernel's per-4-board fp32 loop re-read 2.4 MB
// of weights per role per 4 boards): logits[n][j] = sum_k f[n][k] W[k][j] + b[j], in split
// precision (hi*hi + hi*lo + lo*hi, fp32 accumulation) whatever the trunk's mode, so the heads stay
// fp32-class.  Grid (board tiles of 64, j-chunks of 128, roles); wave w takes boards
// [64 bx + 16 w, +16) x the WG's 8 j-tiles of 16.  A = packed W^T fragments (row j, 8 k per lane),
// B = the boards' features (col = board, 8 k per lane), split to hi / lo on the fly.
__global__ void __launch_bounds__(256) policy_gemm_kernel(const KParams kp) {
    const int r = blockIdx.z, P = kp.P[r], K = 2 * kp.npos;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int jt0 = blockIdx.y * 8;
    const int njt = (P + 15) / 16;
    if (jt0 >= njt) return;
    const int board = blockIdx.x * 64 + wave * 16 + (lane & 15);
    const int kq = 8 * (lane >> 4);
    const float* f = kp.feat + (size_t)(board < kp.n ? board : 0) * kp.FS + (size_t)r * K;
    f32x4 acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16x8* wp = (const bf16x8*)kp.pdp[r];
    for (int kt = 0; kt < kp.pkt; ++kt) {
        // B: this lane's 8 features (k = 32 kt + kq ..), zero past K or past the launch
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 32 * kt + kq + e;
            x[e] = (board < kp.n && k < K) ? f[k] : 0.f;
        }
        bf16x8 bh, bl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            bh[e] = (__bf16)x[e];
            bl[e] = (__bf16)(x[e] - (float)bh[e]);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int jt = jt0 + t;
            if (jt < njt) {
                const size_t o = ((size_t)jt * kp.pkt + kt) * 128 + lane;   // [jt][kt][part][lane]
                const bf16x8 ah = wp[o], al = wp[o + 64];
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[t], 0, 0, 0);
            }
        }
    }
    if (board >= kp.n) return;
    int lof = 0;
    for (int q = 0; q < r; ++q) lof += kp.P[q];
    float* out = kp.glog + (size_t)board * kp.plog + lof;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int j0 = (jt0 + t) * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (j0 + i < P) out[j0 + i] = acc[t][i] + kp.pb[r][j0 + i];
    }
}

__global__ void __launch_bounds__(256) heads_kernel(const KParams kp) {
    constexpr int BPW = kHeadBoards;
    extern __shared__ __attribute__((aligned(16))) float hs[];
    const int FS = kp.FS;
    float* fk = hs;                       // [FS][BPW]
    float* lg = hs + FS * BPW;            // [BPW][LMAX]
    const int tid = threadIdx.x;
    const int board0 = blockIdx.x * BPW;
    const int nb = kp.n - board0 < BPW ? kp.n - board0 : BPW;
    // the boards' features, 8 loads per thread in flight per round (not one load / store at a time)
    for (int i0 = 0; i0 < BPW * FS; i0 += 8 * 256) {
        float r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + tid;
            const int b = i / FS, k = i - b * FS;
            r[u] = (i < BPW * FS && b < nb) ? kp.feat[(size_t)(board0 + b) * FS + k] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + tid;
            const int b = i / FS, k = i - b * FS;
            if (i < BPW * FS) fk[k * BPW + b] = r[u];
        }
    }
    __syncthreads();
    dense_heads<BPW>(kp, fk, lg, board0, nb);
}

#endif

__host__ inline int heads_lds_bytes(int FS, int lgrow) {
    return (FS * kHeadBoards + kHeadBoards * lgrow + kHeadBoards * 4) * 4;
}

}  // namespace gznn
