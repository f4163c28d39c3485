// libgz_nn.so -- C-ABI (include/gzero_nn.h) around the fused gfx950 forward kernel.
//
// Host side: parses the canonical Keras-order float32 blob (galvanise_zero_amd/nn/desc.py
// weight_spec), folds inference BatchNorm (eps 1e-3, model.py:21-22) into the preceding conv,
// packs conv kernels into bf16 MFMA fragment order and uploads one device allocation.
#define GZNN_DEFINE_HEADS_KERNEL
#include "forward_kernel.h"
#include "trunk_variants.h"
#include "../../../include/gzero_nn.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace gznn;

static thread_local std::string g_err;

static int fail(const std::string& msg) {
    g_err = msg;
    return -1;
}

#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)


struct gz_net {
    gz_net_desc d;
    int device = 0;
    int K0 = 0;
    size_t nweights = 0;
    struct Trunk {
        const void* fn = nullptr;
        int nb = 1;                // boards per workgroup
        int smem = 0;              // dynamic LDS bytes
        int btab_off = 0;          // LDS offset of the bias table
        int se_off = 0;            // LDS offset of the squeeze-excite scratch
        int cal_off = 0;           // LDS offset of the concat_all_layers partial sums
        bool fused_heads = false;  // the dense heads run inside the trunk kernel (no heads_kernel launch)
        int resid_bytes = 0;       // global residual scratch per workgroup
        int threads = 256;         // workgroup size (512: two wave groups)
        std::string name;          // kernel name (rocprofv3's)
    } small, large;                // launches below / from large_min_rows rows
    int large_min_rows = 1 << 30;
    int p2 = 1;                    // bf16 parts per operand: 1 (bf16) or 2 (split precision)
    int fpad = 0;                  // filters rounded up to the compiled 64 / 128 / 256 (zero channels)
    bool has_weights = false;
    size_t image_bytes = 0;        // bytes of the device weight image
    float last_roll_ms = 0.f;      // device time of the last gz_net_set_weights_device

    char* dmem = nullptr;          // all weights, one allocation
    KParams kp{};                  // weight pointers filled in, outputs per launch
    std::mutex wmu;                // guards dmem / kp's weight pointers / has_weights (weight rolls)

    hipStream_t stream = nullptr;  // for the synchronous host-buffer forward
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float* d_io = nullptr;         // staging: planes + outputs
    int io_cap = 0;
    float last_ms = 0.f;
    int heads_smem = 0;
    bool gemm_heads = false;       // policy heads by policy_gemm_kernel (single-image nets, large P)
    std::map<hipStream_t, std::pair<float*, int>> glog;   // its logits scratch per stream
    std::mutex feat_mu;            // head-feature scratch, one per stream (launches on one stream are ordered)
    std::map<hipStream_t, std::pair<float*, int>> feat;
    std::map<hipStream_t, std::pair<char*, size_t>> resid;   // global-residual scratch per stream
    unsigned long long* d_stamps = nullptr;   // GZ_KERNEL_STAMPS diagnostics
    int stamp_cap = 0;
    bool stamps_on = false;
    double stamp_avg[8] = {0};
};

extern "C" const char* gz_nn_last_error(void) { return g_err.c_str(); }

// ---- kernel instantiations: trunk_variants.h (per padded filter count and position tiles) ----------
// Variants: NB = boards per workgroup (weight-fragment reuse factor), WPE = minimum resident waves
// per SIMD the register budget must allow (= workgroups per CU).  GZ_KERNEL_VARIANT=<NB><WPE>
// (e.g. "12") overrides the per-launch choice for experiments.

// Measured on MI355X (profiles/r01c_kernel_variants.txt): one board per workgroup with the whole
// register file (11) is fastest while the launch has fewer boards than ~1.5x the CU count; from
// there two boards per workgroup (21) win, each weight fragment feeding twice the MFMAs.  Every
// variant computes each row identically (tests/test_nn_gpu.py::test_kernel_variants_identical), so
// choosing per launch keeps results batch-invariant.
// Launches of 257-383 rows also take the two-board kernel: at one board per workgroup they would
// need a second wave of workgroups on the 256 CUs (one trunk workgroup per CU by LDS).
// large launches: the two-board 4-wave kernel (21).  The 8-wave kernel (24) is 5 % faster back to
// back (profiles/r04t_w8_kexp.txt) but equal inside the bench, whose launches arrive with gaps
// (0.4954 vs 0.4942 ms per 1,024-row launch, same box; profiles/r04x_variants_in_bench.txt):
// selectable (GZ_KERNEL_VARIANT=24), bit-identical.  Round 5: the split F = 128 kernels of boards up
// to 64 positions take variant 23 (trunk_kernel_h2: two groups of two waves, a board each -- half the
// B-fragment reads per MFMA), 1-1.5 % faster than 21 at 1,024 rows (profiles/r05t_ab_v23.txt) and
// bit-identical (the kernels build with -ffp-contract=on).  kLargeFallback: where kLargeVariant is
// not compiled for a geometry.
constexpr int kSmallVariant = 11, kLargeVariant = 23, kLargeFallback = 21, kLargeMinRows = 257;
constexpr int kCUs = 256;

static KernelChoice select_kernel(int fpad, int pt, int v, int precision, bool v2) {
    if (pt < 1 || pt > kMaxPT) return KernelChoice{};
    return trunk_variant(fpad, pt, v, precision, v2);
}

// ---- bf16 (round to nearest even) -------------------------------------------------------------
static inline __host__ __device__ uint16_t f2bf(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// Element offset (within one trunk conv's image) of weight [co][ci] of tap `tap`, hi part; the lo
// part (split precision) sits 512 elements (1 KB) further.  A k-step (tap, 32 input channels) is
// FP/16 blocks of 16 output channels; block = P2 fragments of 1 KB, each in MFMA A-fragment lane
// order (lane = co % 16 + 16 * (k / 8), 8 consecutive k per lane), so one wave-wide 16-byte load
// reads 1 KB contiguous (forward_kernel.h FragOff).
static inline __host__ __device__ size_t wres_index(int tap, int co, int ci, int FP, int P2) {
    const int kc = ci >> 5, k = ci & 31;
    const size_t blk = ((size_t)(tap * (FP >> 5) + kc) * (FP >> 4) + (co >> 4)) * P2;
    return (blk * 64 + (co & 15) + 16 * (k >> 3)) * 8 + (k & 7);
}

static int initial_kernel(const gz_net_desc& d) {
    return d.initial_kernel ? d.initial_kernel : (d.resnet_v2 ? 1 : d.cnn_kernel_size);
}
static bool has_initial_bn(const gz_net_desc& d) { return !d.resnet_v2 || d.initial_bn; }
static int gap_features(const gz_net_desc& d) { return d.global_pooling_value ? d.cnn_filter_size : 0; }
// trunk layers the concat_all_layers value head reads (model.py:251-260), 0 for the other heads
static int cal_layers(const gz_net_desc& d) { return d.concat_all_layers ? d.residual_layers + 1 : 0; }
// value hidden Dense inputs
static int value_features(const gz_net_desc& d) {
    const int HW = d.input_columns * d.input_rows;
    return d.concat_all_layers ? cal_layers(d) * HW : gap_features(d) + HW;
}

// float count of the canonical blob: galvanise_zero_amd/nn/desc.py weight_spec
static size_t spec_count(const gz_net_desc& d) {
    const size_t F = d.cnn_filter_size, C = d.input_channels, k = d.cnn_kernel_size, k0 = initial_kernel(d);
    const size_t HW = (size_t)d.input_columns * d.input_rows, cb = d.conv_bias ? 1 : 0;
    size_t n = k0 * k0 * C * F + cb * F + (has_initial_bn(d) ? 4 * F : 0);
    const size_t conv = k * k * F * F + cb * F;
    const size_t blk = d.resnet_v2 ? 4 * F + conv + 4 * F + conv + 2 * F * (size_t)d.se_units : 2 * (conv + 4 * F);
    n += (size_t)d.residual_layers * blk;
    for (int r = 0; r < d.role_count; ++r) n += F * 2 + cb * 2 + 4 * 2 + 2 * HW * d.policy_dist_count[r] + d.policy_dist_count[r];
    if (d.concat_all_layers) n += (size_t)cal_layers(d) * (F + cb + 4);   // a conv + BN per trunk layer
    else n += F + cb + (d.value_bn ? 4 : 0);
    n += (size_t)value_features(d) * d.value_hidden_size + d.value_hidden_size + (size_t)d.value_hidden_size * d.num_values +
         d.num_values;
    return n;
}

extern "C" gz_net* gz_net_create(const gz_net_desc* desc, int device) {
    if (!desc) { fail("null desc"); return nullptr; }
    const gz_net_desc& d = *desc;
    if (d.cnn_kernel_size != 3) { fail("only cnn_kernel_size 3 is supported"); return nullptr; }
    if (d.role_count < 1 || d.role_count > GZ_MAX_ROLES) { fail("role_count out of range"); return nullptr; }
    if (d.num_values < 1 || d.num_values > 4) { fail("num_values out of range"); return nullptr; }
    if (initial_kernel(d) != 1 && initial_kernel(d) != 3) { fail("initial conv kernel must be 1 or 3"); return nullptr; }
    if (d.se_units < 0 || d.se_units > kMaxSE || (d.se_units && !d.resnet_v2)) {
        fail("squeeze-excite units must be 0.." + std::to_string(kMaxSE) + " on a v2 net");
        return nullptr;
    }
    if (d.concat_all_layers && (!d.resnet_v2 || d.global_pooling_value || d.value_bn)) {
        fail("concat_all_layers needs a v2 net without the pooling value head (model.py:251-252)");
        return nullptr;
    }
    const int precision = d.precision == 0 ? GZ_PRECISION_BF16 : d.precision;
    if (precision != GZ_PRECISION_BF16 && precision != GZ_PRECISION_SPLIT) { fail("unknown precision"); return nullptr; }
    int vs = kSmallVariant, vl = kLargeVariant, min_large = kLargeMinRows;
    if (const char* e = getenv("GZ_KERNEL_VARIANT")) {   // experiments: one fixed variant
        vs = vl = atoi(e);
        min_large = 1 << 30;
    }
    // kernels are compiled per padded filter count and position-tile count; the board's H and W
    // are kernel arguments (H = input_columns, W = input_rows: bases.py:104-121)
    const int npos_ = d.input_columns * d.input_rows;
    const int pt = kernel_tiles((npos_ + 15) / 16);
    const int fpad = kernel_filters(d.cnn_filter_size, (npos_ + 15) / 16);
    if (d.input_rows > 32 || npos_ >= 1024) { fail("board too large"); return nullptr; }
    const bool v2 = d.resnet_v2 != 0;
    KernelChoice kc = select_kernel(fpad, pt, vs, precision, v2);
    KernelChoice kl = select_kernel(fpad, pt, vl, precision, v2);
    if (!kl.fn && vl == kLargeVariant) kl = select_kernel(fpad, pt, kLargeFallback, precision, v2);
    // wave-group kernels: each group's staging / heads scratch must fit its own image
    auto wg_fits = [&](const KernelChoice& c) {
        if (c.groups == 1) return true;
        const int np = d.input_columns * d.input_rows;
        int mp = 0;
        for (int r = 0; r < d.role_count; ++r) mp = std::max(mp, d.policy_dist_count[r]);
        const int kk0 = initial_kernel(d);
        const int k0p = ((kk0 * kk0 * d.input_channels + 31) / 32) * 32;
        const int p2 = precision == GZ_PRECISION_SPLIT ? 2 : 1;
        (void)mp;
        return trunk_scratch_bytes(np, d.input_channels, k0p, d.role_count, p2, fpad) <= c.act_bytes &&
               fused_heads_bytes(np, d.role_count, heads_row(d.role_count, d.policy_dist_count, d.value_hidden_size),
                                 gap_features(d), c.nb, 1, fpad) <= c.act_bytes;
    };
    if (kl.fn && !wg_fits(kl)) {
        // the wave-group default (23) does not fit this geometry's scratch: the two-board 4-wave
        // kernel (21, one image per workgroup) before the one-board one
        kl = vl == kLargeVariant ? select_kernel(fpad, pt, kLargeFallback, precision, v2) : KernelChoice{};
        if (kl.fn && !wg_fits(kl)) kl = KernelChoice{};
    }
    if (kc.fn && !wg_fits(kc)) kc = KernelChoice{};
    if (kc.fn && !kl.fn && vl != vs) {   // geometries with a single (one board per workgroup) variant
        kl = kc;
        min_large = 1 << 30;
    }
    if (!kc.fn || !kl.fn) {
        fail("unsupported network geometry F=" + std::to_string(d.cnn_filter_size) + " H=" +
             std::to_string(d.input_columns) + " W=" + std::to_string(d.input_rows) +
             (precision == GZ_PRECISION_SPLIT ? " (split precision)" : "") + (v2 ? " (v2 nets: F <= 128)" : ""));
        return nullptr;
    }
    gz_net* net = new gz_net;
    net->d = d;
    net->device = device;
    net->large_min_rows = min_large;
    net->p2 = precision == GZ_PRECISION_SPLIT ? 2 : 1;
    net->fpad = fpad;
    const int k0 = initial_kernel(d);
    net->K0 = ((k0 * k0 * d.input_channels + 31) / 32) * 32;
    net->nweights = spec_count(d);
    int maxP = 0;
    for (int r = 0; r < d.role_count; ++r) maxP = std::max(maxP, d.policy_dist_count[r]);
    const int npos = d.input_columns * d.input_rows;
    // the dense heads' LDS row: the two-phase layout where every kernel's LDS still fits, else the
    // sequential one (forward_kernel.h dense_heads / dense_heads_seq)
    int lgrow = heads_row(d.role_count, d.policy_dist_count, d.value_hidden_size, true);
    bool heads_seq = false;
    // LDS: two ping-pong activation images per board; the scratch (input staging, heads) aliases
    // the second image set, which holds nothing live at those times.
    const int scr_in = trunk_scratch_bytes(npos, d.input_channels, net->K0, d.role_count, net->p2, fpad);
    auto trunk = [&](const KernelChoice& c) {
        gz_net::Trunk t;
        t.fn = c.fn;
        t.nb = c.nb;
        t.threads = c.threads;
        t.name = c.name;
        t.fused_heads = !c.single_image && !d.concat_all_layers;
        const int scr = t.fused_heads ? std::max(scr_in, fused_heads_bytes(npos, d.role_count, lgrow, gap_features(d), c.nb,
                                                                           c.groups == 2 ? 1 : c.nb, fpad))
                                      : scr_in;
        t.btab_off = c.single_image ? align16(std::max(c.act_bytes, scr))
                                    : c.nb * c.act_bytes + std::max(c.nb * c.act_bytes, scr);
        t.resid_bytes = c.resid_bytes;
        t.smem = t.btab_off + bias_table_bytes(fpad, d.residual_layers);
        t.se_off = t.smem;
        if (d.se_units) t.smem += se_scratch_bytes(fpad, c.nb);
        t.cal_off = t.smem;
        if (d.concat_all_layers) t.smem += align16(4 * c.nb * npos * 4);
        return t;
    };
    const int FS = 2 * d.role_count * npos + value_features(d);   // head features per board
    for (int pass = 0; pass < 2; ++pass) {
        net->small = trunk(kc);
        net->large = trunk(kl);
        net->heads_smem = heads_lds_bytes(FS, lgrow);
        if (pass == 1 || (net->small.smem <= 160 * 1024 && net->large.smem <= 160 * 1024 && net->heads_smem <= 160 * 1024))
            break;
        heads_seq = true;
        lgrow = heads_row(d.role_count, d.policy_dist_count, d.value_hidden_size, false);
    }
    // Large policies on nets whose every launch runs the separate heads kernel: the policy Dense
    // layers run as one MFMA GEMM per launch (policy_gemm_kernel) instead of heads_kernel's
    // per-4-board fp32 loop (amazons P = 3041: 12 % of the forward).  Every launch of such a net
    // takes this path, so results stay batch-invariant.
    net->gemm_heads = !net->small.fused_heads && !net->large.fused_heads && maxP >= 512 &&
                      getenv("GZ_NO_GEMM_HEADS") == nullptr;
    KParams& kp = net->kp;
    kp.C = d.input_channels;
    kp.K0 = net->K0;
    kp.B = d.residual_layers;
    kp.R = d.role_count;
    kp.VH = d.value_hidden_size;
    kp.V = d.num_values;
    kp.leaky = d.leaky_relu;
    kp.flatten_nchw = d.flatten_nchw;
    kp.value_sigmoid = d.value_sigmoid;
    kp.v2 = d.resnet_v2 ? 1 : 0;
    kp.k0taps = k0 * k0;
    kp.init_act = has_initial_bn(d) ? 1 : 0;
    kp.S = d.se_units;
    kp.gapF = gap_features(d);
    kp.FS = FS;
    kp.VK = value_features(d);
    kp.cal = cal_layers(d);
    kp.nofuse = d.concat_all_layers ? 1 : 0;
    kp.maxP = maxP;
    kp.lgrow = lgrow;
    kp.heads_seq = heads_seq ? 1 : 0;
    kp.npos = npos;
    kp.gemm_heads = net->gemm_heads ? 1 : 0;
    kp.pkt = (2 * npos + 31) / 32;
    kp.plog = 0;
    for (int r = 0; r < d.role_count; ++r) kp.plog += d.policy_dist_count[r];
    kp.H = d.input_columns;
    kp.W = d.input_rows;
    kp.wmagic = (65536 + kp.W - 1) / kp.W;
    for (int r = 0; r < d.role_count; ++r) kp.P[r] = d.policy_dist_count[r];

    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&net->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&net->ev0) != hipSuccess || hipEventCreate(&net->ev1) != hipSuccess) {
        fail(std::string("HIP init failed: ") + hipGetErrorString(hipGetLastError()));
        delete net;
        return nullptr;
    }
    for (const gz_net::Trunk* t : {&net->small, &net->large}) {
        if (t->smem > 160 * 1024) {
            fail("network needs " + std::to_string(t->smem) + " B of LDS per workgroup (160 KB max)");
            delete net;
            return nullptr;
        }
        if (t->smem > 64 * 1024 &&
            hipFuncSetAttribute(t->fn, hipFuncAttributeMaxDynamicSharedMemorySize, t->smem) != hipSuccess) {
            fail("cannot raise dynamic LDS limit");
            delete net;
            return nullptr;
        }
    }
    if (net->heads_smem > 64 * 1024 &&
        hipFuncSetAttribute((const void*)&heads_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, net->heads_smem) !=
            hipSuccess) {
        fail("cannot raise dynamic LDS limit (heads)");
        delete net;
        return nullptr;
    }
    return net;
}

extern "C" void gz_net_destroy(gz_net* net) {
    if (!net) return;
    (void)hipSetDevice(net->device);
    if (net->dmem) (void)hipFree(net->dmem);
    if (net->d_io) (void)hipFree(net->d_io);
    if (net->d_stamps) (void)hipFree(net->d_stamps);
    for (auto& f : net->feat) (void)hipFree(f.second.first);
    for (auto& f : net->resid) (void)hipFree(f.second.first);
    for (auto& f : net->glog) (void)hipFree(f.second.first);
    if (net->ev0) (void)hipEventDestroy(net->ev0);
    if (net->ev1) (void)hipEventDestroy(net->ev1);
    if (net->stream) (void)hipStreamDestroy(net->stream);
    delete net;
}

extern "C" size_t gz_net_weight_count(const gz_net* net) { return net ? net->nweights : 0; }

extern "C" int gz_net_heads_fused(const gz_net* net) { return net->large.fused_heads ? 1 : 0; }

extern "C" double gz_net_flops_per_eval(const gz_net* net) {
    const gz_net_desc& d = net->d;   // = NetDesc.flops_per_eval (desc.py)
    const double F = d.cnn_filter_size, C = d.input_channels, HW = (double)d.input_columns * d.input_rows;
    const double k0 = initial_kernel(d);
    double f = 2 * HW * C * F * k0 * k0 + d.residual_layers * 2 * (2 * HW * F * F * 9);
    f += d.residual_layers * 2.0 * (2 * F * d.se_units);
    for (int r = 0; r < d.role_count; ++r) f += 2 * HW * F * 2 + 2 * (2 * HW) * d.policy_dist_count[r];
    f += 2 * HW * F * std::max(1, cal_layers(d)) + 2.0 * value_features(d) * d.value_hidden_size +
         2.0 * d.value_hidden_size * d.num_values;
    return f;
}

// ---- weight folding / packing ---------------------------------------------------------------
namespace {
struct Cursor {
    const float* p;
    const float* take(size_t n) { const float* r = p; p += n; return r; }
};

struct Layout {
    size_t off = 0;
    size_t alloc(size_t bytes) { size_t o = off; off = (off + bytes + 255) & ~(size_t)255; return o; }
};

// The device weight image: byte offsets of every packed tensor (one allocation), the same for the
// host packing (gz_net_set_weights) and the device one (gz_net_set_weights_device)
struct ImageLayout {
    size_t w0, w0lo, b0, wres, bres, wh, bh, wcl, bcl, pd[GZ_MAX_ROLES], pb[GZ_MAX_ROLES], vhw, vhb, pre, sew1, sew2, vdw,
        vdb, pdp[GZ_MAX_ROLES] = {}, total;
    // element counts
    size_t n_w0, n_wres, n_wh, n_wcl, n_pd[GZ_MAX_ROLES], n_vhw, n_pre, n_sew1, n_sew2, n_pdp[GZ_MAX_ROLES] = {};
};

ImageLayout image_layout(const gz_net* net) {
    const gz_net_desc& d = net->d;
    const int FP = net->fpad, B = d.residual_layers, R = d.role_count, P2 = net->p2, S = d.se_units;
    const int HW = d.input_columns * d.input_rows, HC = 2 * R + 1, NL = cal_layers(d);
    const int VH = d.value_hidden_size, VK = value_features(d);
    ImageLayout I;
    I.n_w0 = (size_t)net->K0 * FP;
    I.n_wres = (size_t)P2 * 2 * B * 9 * FP * FP;
    I.n_wh = (size_t)HC * FP;
    I.n_wcl = (size_t)std::max(NL, 1) * FP;
    for (int r = 0; r < R; ++r) I.n_pd[r] = (size_t)2 * HW * ((d.policy_dist_count[r] + 3) & ~3);
    I.n_vhw = (size_t)VK * ((VH + 3) & ~3);
    I.n_pre = d.resnet_v2 ? (size_t)2 * B * FP : 1;
    I.n_sew1 = S ? (size_t)B * FP * S : 1;
    I.n_sew2 = S ? (size_t)B * S * FP : 1;
    Layout L;
    I.w0 = L.alloc(I.n_w0 * 2);
    I.w0lo = L.alloc((P2 == 2 ? I.n_w0 : 1) * 2);
    I.b0 = L.alloc((size_t)FP * 4);
    I.wres = L.alloc(I.n_wres * 2);
    I.bres = L.alloc((size_t)2 * B * FP * 4);
    I.wh = L.alloc(I.n_wh * 4);
    I.bh = L.alloc((size_t)HC * 4);
    I.wcl = L.alloc(I.n_wcl * 4);
    I.bcl = L.alloc((size_t)std::max(NL, 1) * 4);
    for (int r = 0; r < R; ++r) {
        I.pd[r] = L.alloc(I.n_pd[r] * 4);
        I.pb[r] = L.alloc((size_t)d.policy_dist_count[r] * 4);
    }
    I.vhw = L.alloc(I.n_vhw * 4);
    I.vhb = L.alloc((size_t)VH * 4);
    I.pre = L.alloc(I.n_pre * 4);
    I.sew1 = L.alloc(I.n_sew1 * 4);
    I.sew2 = L.alloc(I.n_sew2 * 4);
    I.vdw = L.alloc((size_t)VH * d.num_values * 4);
    I.vdb = L.alloc((size_t)d.num_values * 4);
    if (net->gemm_heads) {
        const int nkt = (2 * HW + 31) / 32;
        for (int r = 0; r < R; ++r) {
            I.n_pdp[r] = (size_t)((d.policy_dist_count[r] + 15) / 16) * nkt * 2 * 64 * 8;
            I.pdp[r] = L.alloc(I.n_pdp[r] * 2);
        }
    }
    I.total = L.off;
    return I;
}

// Swaps in the device image m (laid out by I) under the lock launch_segments takes, so a launcher
// thread running a generation roll sees either the old or the new image, never a mix; the replaced
// image is freed after a device sync (launches already queued may still read it).
int install_image(gz_net* net, char* m, const ImageLayout& I) {
    const int R = net->d.role_count;
    std::unique_lock<std::mutex> wl(net->wmu);
    char* old = net->dmem;
    net->dmem = m;
    KParams& kp = net->kp;
    kp.w0 = (const __bf16*)(m + I.w0);
    kp.w0lo = (const __bf16*)(m + I.w0lo);
    kp.b0 = (const float*)(m + I.b0);
    kp.wres = (const __bf16*)(m + I.wres);
    kp.bres = (const float*)(m + I.bres);
    kp.wh = (const float*)(m + I.wh);
    kp.bh = (const float*)(m + I.bh);
    kp.wcl = (const float*)(m + I.wcl);
    kp.bcl = (const float*)(m + I.bcl);
    for (int r = 0; r < R; ++r) {
        kp.pd[r] = (const float*)(m + I.pd[r]);
        kp.pb[r] = (const float*)(m + I.pb[r]);
    }
    kp.vhw = (const float*)(m + I.vhw);
    kp.vhb = (const float*)(m + I.vhb);
    kp.vdw = (const float*)(m + I.vdw);
    kp.vdb = (const float*)(m + I.vdb);
    kp.pre = (const float*)(m + I.pre);
    kp.sew1 = (const float*)(m + I.sew1);
    kp.sew2 = (const float*)(m + I.sew2);
    for (int r = 0; r < R; ++r) kp.pdp[r] = net->gemm_heads ? (const __bf16*)(m + I.pdp[r]) : nullptr;
    net->has_weights = true;
    net->image_bytes = I.total;
    wl.unlock();
    if (old) {
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipFree(old));
    }
    return 0;
}
}  // namespace

extern "C" int gz_net_set_weights(gz_net* net, const float* blob, size_t count) {
    if (!net || !blob) return fail("null argument");
    if (count != net->nweights)
        return fail("weight count mismatch: got " + std::to_string(count) + " expected " + std::to_string(net->nweights));
    const gz_net_desc& d = net->d;
    // F = the model's filters; FP = the kernel's (padded with zero channels: zero weights and zero
    // folded bias keep them at 0 through every ReLU and residual add)
    const int F = d.cnn_filter_size, C = d.input_channels, B = d.residual_layers, R = d.role_count;
    const int FP = net->fpad;
    const int HW = d.input_columns * d.input_rows, K0 = net->K0, KC = FP / 32;
    const int HC = 2 * R + 1;      // head 1x1 convs (the value conv: unused with concat_all_layers)
    const int NL = cal_layers(d);
    const float eps = 1e-3f;

    // host images
    const int P2 = net->p2;
    std::vector<uint16_t> w0((size_t)K0 * FP, 0), w0lo(P2 == 2 ? (size_t)K0 * FP : 0, 0);
    std::vector<float> b0(FP, 0.f);
    std::vector<uint16_t> wres((size_t)P2 * 2 * B * 9 * FP * FP, 0);
    // split precision: x = hi + lo, hi = bf16(x), lo = bf16(x - hi)
    auto lo_of = [](float v) {
        const uint16_t h = f2bf(v);
        uint32_t u = (uint32_t)h << 16;
        float hf;
        std::memcpy(&hf, &u, 4);
        return f2bf(v - hf);
    };
    std::vector<float> bres((size_t)2 * B * FP, 0.f);
    std::vector<float> wh((size_t)HC * FP, 0.f), bh(HC, 0.f);
    std::vector<float> wcl((size_t)std::max(NL, 1) * FP, 0.f), bcl(std::max(NL, 1), 0.f);

    Cursor cur{blob};
    // BN after a conv with bias cb (legacy model files): gamma*(conv + cb - mean)/sqrt(var+eps) + beta
    // = scale*conv + (beta + (cb - mean)*scale)
    auto bn_fold = [&](int n, std::vector<float>& scale, std::vector<float>& bias, const float* cb = nullptr) {
        const float* g = cur.take(n);
        const float* be = cur.take(n);
        const float* mu = cur.take(n);
        const float* var = cur.take(n);
        scale.resize(n);
        bias.resize(n);
        for (int i = 0; i < n; ++i) {
            scale[i] = g[i] / std::sqrt(var[i] + eps);
            bias[i] = cb ? be[i] + (cb[i] - mu[i]) * scale[i] : be[i] - mu[i] * scale[i];
        }
    };
    auto conv_bias = [&](int n) -> const float* { return d.conv_bias ? cur.take(n) : nullptr; };
    std::vector<float> s, bb;
    const int k0 = initial_kernel(d), T0 = k0 * k0, S = d.se_units;
    {   // initial conv [k0][k0][C][F] -> w0[kc][co][32], k = tap*C + c
        const float* w = cur.take((size_t)T0 * C * F);
        const float* cb = conv_bias(F);
        if (has_initial_bn(d)) {
            bn_fold(F, s, bb, cb);
        } else {   // v2 files with a bare initial conv: s = conv (+ bias), no BN, no activation
            s.assign(F, 1.f);
            bb.assign(F, 0.f);
            if (cb) for (int i = 0; i < F; ++i) bb[i] = cb[i];
        }
        for (int co = 0; co < F; ++co) {
            b0[co] = bb[co];
            for (int k = 0; k < T0 * C; ++k) {
                const int tap = k / C, c = k % C;
                const float v = w[((size_t)tap * C + c) * F + co] * s[co];
                w0[((size_t)(k / 32) * FP + co) * 32 + (k % 32)] = f2bf(v);
                if (P2 == 2) w0lo[((size_t)(k / 32) * FP + co) * 32 + (k % 32)] = lo_of(v);
            }
        }
    }
    // trunk conv `conv` [3][3][F][F] * scale[co] -> wres_index order, bias[co] -> bres
    auto pack_conv = [&](int conv, const float* w, const std::vector<float>& scale, const std::vector<float>& bias) {
        uint16_t* dst = wres.data() + (size_t)P2 * conv * 9 * FP * FP;
        for (int co = 0; co < F; ++co) {
            bres[(size_t)conv * FP + co] = bias[co];
            for (int tap = 0; tap < 9; ++tap)
                for (int ci = 0; ci < F; ++ci) {
                    const float v = w[((size_t)tap * F + ci) * F + co] * scale[co];
                    const size_t o = wres_index(tap, co, ci, FP, P2);
                    dst[o] = f2bf(v);
                    if (P2 == 2) dst[o + 512] = lo_of(v);
                }
        }
    };
    std::vector<float> pre(d.resnet_v2 ? (size_t)2 * B * FP : 1, 0.f);
    std::vector<float> sew1(S ? (size_t)B * FP * S : 1, 0.f), sew2(S ? (size_t)B * S * FP : 1, 0.f);
    for (int blk = 0; blk < B; ++blk) {
        if (!d.resnet_v2) {      // conv-BN-act-conv-BN-add-act: both BNs fold into their convs
            for (int j = 0; j < 2; ++j) {
                const float* w = cur.take((size_t)9 * F * F);
                const float* cb = conv_bias(F);
                bn_fold(F, s, bb, cb);
                pack_conv(2 * blk + j, w, s, bb);
            }
            continue;
        }
        // v2: BN_1 (scale / shift applied to the stream when the block's input image is written),
        // conv1 with BN_2 folded, conv2 (no BN), squeeze-excite dense layers
        bn_fold(F, s, bb);
        for (int co = 0; co < F; ++co) {
            pre[(size_t)(2 * blk) * FP + co] = s[co];
            pre[(size_t)(2 * blk + 1) * FP + co] = bb[co];
        }
        const float* w1 = cur.take((size_t)9 * F * F);
        const float* cb1 = conv_bias(F);
        bn_fold(F, s, bb, cb1);
        pack_conv(2 * blk, w1, s, bb);
        const float* w2 = cur.take((size_t)9 * F * F);
        const float* cb2 = conv_bias(F);
        std::vector<float> one(F, 1.f), b2(F, 0.f);
        if (cb2) for (int co = 0; co < F; ++co) b2[co] = cb2[co];
        pack_conv(2 * blk + 1, w2, one, b2);
        if (S) {
            const float* c = cur.take((size_t)F * S);   // Dense [F][S]
            const float* gt = cur.take((size_t)S * F);  // Dense [S][F]
            for (int ci = 0; ci < F; ++ci)
                for (int j = 0; j < S; ++j) sew1[((size_t)blk * FP + ci) * S + j] = c[(size_t)ci * S + j];
            for (int j = 0; j < S; ++j)
                for (int co = 0; co < F; ++co) sew2[((size_t)blk * S + j) * FP + co] = gt[(size_t)j * F + co];
        }
    }
    std::vector<const float*> pdense(R), pbias(R);
    for (int r = 0; r < R; ++r) {
        const float* w = cur.take((size_t)F * 2);   // [1][1][F][2]
        const float* cb = conv_bias(2);
        bn_fold(2, s, bb, cb);
        for (int c = 0; c < 2; ++c) {
            for (int f = 0; f < F; ++f) wh[(size_t)(2 * r + c) * FP + f] = w[(size_t)f * 2 + c] * s[c];
            bh[2 * r + c] = bb[c];
        }
        pdense[r] = cur.take((size_t)2 * HW * d.policy_dist_count[r]);
        pbias[r] = cur.take(d.policy_dist_count[r]);
    }
    for (int j = 0; j < NL; ++j) {   // concat_all_layers: conv2d_block(1, 1) per trunk layer, BN folded
        const float* w = cur.take(F);
        const float* cb = conv_bias(1);
        bn_fold(1, s, bb, cb);
        for (int f = 0; f < F; ++f) wcl[(size_t)j * FP + f] = w[f] * s[0];
        bcl[j] = bb[0];
    }
    if (NL == 0) {
        const float* w = cur.take(F);   // [1][1][F][1], no BN, no bias (model.py:275-279)
        const float* cb = conv_bias(1);  // legacy files: bias, then BN (value_bn)
        float vs = 1.f, vb = cb ? cb[0] : 0.f;
        if (d.value_bn) {
            bn_fold(1, s, bb, cb);
            vs = s[0];
            vb = bb[0];
        }
        for (int f = 0; f < F; ++f) wh[(size_t)(2 * R) * FP + f] = w[f] * vs;
        bh[2 * R] = vb;
    }
    const int VK = value_features(d);       // value hidden inputs: [GAP F] + HW, or (B + 1) HW
    const float* vhw = cur.take((size_t)VK * d.value_hidden_size);
    const float* vhb = cur.take(d.value_hidden_size);
    const float* vdw = cur.take((size_t)d.value_hidden_size * d.num_values);
    const float* vdb = cur.take(d.num_values);
    if ((size_t)(cur.p - blob) != count) return fail("internal: blob cursor mismatch");

    // the dense heads' weights with their output dimension padded to a multiple of 4 ([K][N4], zero
    // columns: forward_kernel.h dense_heads loads 4 consecutive outputs per float4)
    auto pad4 = [](const float* w, int K, int N) {
        const int N4 = (N + 3) & ~3;
        std::vector<float> q((size_t)K * N4, 0.f);
        for (int k = 0; k < K; ++k) std::memcpy(q.data() + (size_t)k * N4, w + (size_t)k * N, (size_t)N * 4);
        return q;
    };
    std::vector<std::vector<float>> pdq(R);
    for (int r = 0; r < R; ++r) pdq[r] = pad4(pdense[r], 2 * HW, d.policy_dist_count[r]);
    const std::vector<float> vhq = pad4(vhw, VK, d.value_hidden_size);

    // device layout (image_layout: the same offsets as the device packing's)
    const ImageLayout I = image_layout(net);
    // policy_gemm_kernel's A fragments: W^T tiles [jt][kt][hi | lo][64 lanes][8 k] bf16, lane l holding
    // row j = 16 jt + l % 16 and k = 32 kt + 8 (l / 16) + e (zero padded)
    std::vector<std::vector<uint16_t>> pdp(R);
    if (net->gemm_heads) {
        const int K = 2 * HW, nkt = (K + 31) / 32;
        for (int r = 0; r < R; ++r) {
            const int P = d.policy_dist_count[r], njt = (P + 15) / 16;
            pdp[r].assign((size_t)njt * nkt * 2 * 64 * 8, 0);
            for (int jt = 0; jt < njt; ++jt)
                for (int kt = 0; kt < nkt; ++kt)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e) {
                            const int j = 16 * jt + (l & 15), k = 32 * kt + 8 * (l >> 4) + e;
                            if (j >= P || k >= K) continue;
                            const float v = pdense[r][(size_t)k * P + j];
                            const size_t o = ((((size_t)jt * nkt + kt) * 2) * 64 + l) * 8 + e;
                            pdp[r][o] = f2bf(v);
                            pdp[r][o + 64 * 8] = lo_of(v);
                        }
        }
    }

    std::vector<char> img(I.total, 0);
    auto put = [&](size_t off, const void* src, size_t bytes) { std::memcpy(img.data() + off, src, bytes); };
    put(I.w0, w0.data(), w0.size() * 2);
    if (P2 == 2) put(I.w0lo, w0lo.data(), w0lo.size() * 2);
    put(I.b0, b0.data(), b0.size() * 4);
    put(I.wres, wres.data(), wres.size() * 2);
    put(I.bres, bres.data(), bres.size() * 4);
    put(I.wh, wh.data(), wh.size() * 4);
    put(I.bh, bh.data(), bh.size() * 4);
    put(I.wcl, wcl.data(), wcl.size() * 4);
    put(I.bcl, bcl.data(), bcl.size() * 4);
    for (int r = 0; r < R; ++r) {
        put(I.pd[r], pdq[r].data(), pdq[r].size() * 4);   // Keras [2HW][P_r] (k-major), rows padded to P4
        put(I.pb[r], pbias[r], (size_t)d.policy_dist_count[r] * 4);
    }
    put(I.vhw, vhq.data(), vhq.size() * 4);   // Keras [VK][VH], rows padded to VH4
    put(I.pre, pre.data(), pre.size() * 4);
    put(I.sew1, sew1.data(), sew1.size() * 4);
    put(I.sew2, sew2.data(), sew2.size() * 4);
    put(I.vhb, vhb, d.value_hidden_size * 4);
    put(I.vdw, vdw, (size_t)d.value_hidden_size * d.num_values * 4);
    put(I.vdb, vdb, d.num_values * 4);
    if (net->gemm_heads)
        for (int r = 0; r < R; ++r) put(I.pdp[r], pdp[r].data(), pdp[r].size() * 2);

    HIPCHK(hipSetDevice(net->device));
    char* m = nullptr;
    HIPCHK(hipMalloc((void**)&m, I.total));
    if (hipMemcpy(m, img.data(), I.total, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(m);
        return fail("weight upload failed");
    }
    return install_image(net, m, I);
}

// ---- the same packing on the device (generation roll: the blob arrives in HBM by an RCCL broadcast)
// Every value is computed with the host path's operations and rounding (correctly rounded divide /
// sqrt, no contraction, the same bf16 rounding), so the two images are byte-identical
// (tests/test_weight_roll_gpu.py); only the offsets of the blob's tensors are walked on the host.
namespace {
struct BNRef {                  // a BatchNorm over n channels after a conv with optional bias cb
    const float *g = nullptr, *be = nullptr, *mu = nullptr, *var = nullptr, *cb = nullptr;
    int n = 0;                  // g == nullptr: no BN (scale 1, bias cb or 0)
    int out = 0;                // offset of its scale[n] | bias[n] in the fold buffer
};
struct BlobPlan {
    const float* w0 = nullptr;
    BNRef bn0;
    std::vector<const float*> wconv;   // [2B] 3x3 conv kernels
    std::vector<BNRef> bnconv;         // [2B] the BN folded into each
    std::vector<BNRef> pre;            // v2: [B] the block's first BN (scale / shift of the stream)
    std::vector<const float*> se_c, se_g;
    const float* hw[GZ_MAX_ROLES] = {};
    BNRef hbn[GZ_MAX_ROLES];
    const float* pd[GZ_MAX_ROLES] = {};
    const float* pb[GZ_MAX_ROLES] = {};
    std::vector<const float*> clw;
    std::vector<BNRef> clbn;
    const float* vw = nullptr;
    BNRef vbn;
    const float *vhw = nullptr, *vhb = nullptr, *vdw = nullptr, *vdb = nullptr;
    size_t consumed = 0;
    int fold_floats = 0;
};

// the tensors of the canonical blob at base (desc.py weight_spec; the order gz_net_set_weights reads)
BlobPlan blob_plan(const gz_net_desc& d, const float* base) {
    BlobPlan P;
    Cursor cur{base};
    const int F = d.cnn_filter_size, C = d.input_channels, B = d.residual_layers, R = d.role_count, S = d.se_units;
    const int HW = d.input_columns * d.input_rows, k0 = initial_kernel(d), NL = cal_layers(d);
    auto cbias = [&](int n) -> const float* { return d.conv_bias ? cur.take(n) : nullptr; };
    auto bn = [&](int n, const float* cb) {
        BNRef b;
        b.g = cur.take(n); b.be = cur.take(n); b.mu = cur.take(n); b.var = cur.take(n);
        b.cb = cb; b.n = n; b.out = P.fold_floats;
        P.fold_floats += 2 * n;
        return b;
    };
    auto nobn = [&](int n, const float* cb) {
        BNRef b;
        b.cb = cb; b.n = n; b.out = P.fold_floats;
        P.fold_floats += 2 * n;
        return b;
    };
    P.w0 = cur.take((size_t)k0 * k0 * C * F);
    {
        const float* cb = cbias(F);
        P.bn0 = has_initial_bn(d) ? bn(F, cb) : nobn(F, cb);
    }
    for (int blk = 0; blk < B; ++blk) {
        if (!d.resnet_v2) {
            for (int j = 0; j < 2; ++j) {
                P.wconv.push_back(cur.take((size_t)9 * F * F));
                const float* cb = cbias(F);
                P.bnconv.push_back(bn(F, cb));
            }
            continue;
        }
        P.pre.push_back(bn(F, nullptr));
        P.wconv.push_back(cur.take((size_t)9 * F * F));
        {
            const float* cb = cbias(F);
            P.bnconv.push_back(bn(F, cb));
        }
        P.wconv.push_back(cur.take((size_t)9 * F * F));
        P.bnconv.push_back(nobn(F, cbias(F)));
        if (S) {
            P.se_c.push_back(cur.take((size_t)F * S));
            P.se_g.push_back(cur.take((size_t)S * F));
        }
    }
    for (int r = 0; r < R; ++r) {
        P.hw[r] = cur.take((size_t)F * 2);
        const float* cb = cbias(2);
        P.hbn[r] = bn(2, cb);
        P.pd[r] = cur.take((size_t)2 * HW * d.policy_dist_count[r]);
        P.pb[r] = cur.take(d.policy_dist_count[r]);
    }
    for (int j = 0; j < NL; ++j) {
        P.clw.push_back(cur.take(F));
        const float* cb = cbias(1);
        P.clbn.push_back(bn(1, cb));
    }
    if (NL == 0) {
        P.vw = cur.take(F);
        const float* cb = cbias(1);
        P.vbn = d.value_bn ? bn(1, cb) : nobn(1, cb);
    }
    P.vhw = cur.take((size_t)value_features(d) * d.value_hidden_size);
    P.vhb = cur.take(d.value_hidden_size);
    P.vdw = cur.take((size_t)d.value_hidden_size * d.num_values);
    P.vdb = cur.take(d.num_values);
    P.consumed = (size_t)(cur.p - base);
    return P;
}

// Float operations with the host's rounding whatever the device compiler contracts or approximates:
// each computed in double and rounded to float at once -- correctly rounded, since 53 >= 2 x 24 + 2
// bits makes the double rounding innocuous for + - * / sqrt.  The opaque register barriers keep the
// compiler from narrowing the double operation back to a float one and from fusing a multiply with
// the next add into one v_fma_f32 (which -ffp-contract=fast would otherwise do: observed as 1-5 ulp
// differences of the folded biases from the host's).
__device__ __forceinline__ double f_keep(double x) { asm volatile("" : "+v"(x)); return x; }
__device__ __forceinline__ float f_keep(float x) { asm volatile("" : "+v"(x)); return x; }
__device__ __forceinline__ float f_mul(float a, float b) { return f_keep((float)f_keep((double)a * (double)b)); }
__device__ __forceinline__ float f_add(float a, float b) { return f_keep((float)f_keep((double)a + (double)b)); }
__device__ __forceinline__ float f_sub(float a, float b) { return f_keep((float)f_keep((double)a - (double)b)); }
__device__ __forceinline__ float f_div(float a, float b) { return f_keep((float)f_keep(__ddiv_rn((double)a, (double)b))); }
__device__ __forceinline__ float f_sqrt(float a) { return f_keep((float)f_keep(__dsqrt_rn((double)a))); }

__device__ __forceinline__ uint16_t lo_of_dev(float v) {
    const uint16_t h = f2bf(v);
    return f2bf(f_sub(v, __builtin_bit_cast(float, (uint32_t)h << 16)));
}

struct BNJob {
    const float *g, *be, *mu, *var, *cb;
    int n, out;
};
// scale = g / sqrt(var + eps), bias = be - mu scale (with a conv bias: be + (cb - mu) scale); no BN:
// scale 1, bias cb or 0 -- gz_net_set_weights' bn_fold, operation for operation
__global__ void bn_fold_kernel(const BNJob* jobs, float* fold) {
    const BNJob j = jobs[blockIdx.x];
    for (int i = threadIdx.x; i < j.n; i += blockDim.x) {
        float sc = 1.f, bi = j.cb ? j.cb[i] : 0.f;
        if (j.g) {
            sc = f_div(j.g[i], f_sqrt(f_add(j.var[i], 1e-3f)));
            bi = j.cb ? f_add(j.be[i], f_mul(f_sub(j.cb[i], j.mu[i]), sc)) : f_sub(j.be[i], f_mul(j.mu[i], sc));
        }
        fold[j.out + i] = sc;
        fold[j.out + j.n + i] = bi;
    }
}

// one trunk conv [3][3][F][F] * scale[co] -> wres_index order, bf16 (+ its bias row)
__global__ void pack_conv_kernel(const float* w, const float* scale, const float* bias, uint16_t* dst, float* bres,
                                 int F, int FP, int P2) {
    const size_t n = (size_t)9 * F * F;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int co = (int)(i % F), ci = (int)((i / F) % F), tap = (int)(i / ((size_t)F * F));
        const float v = f_mul(w[i], scale[co]);
        const size_t o = wres_index(tap, co, ci, FP, P2);
        dst[o] = f2bf(v);
        if (P2 == 2) dst[o + 512] = lo_of_dev(v);
        if (tap == 0 && ci == 0) bres[co] = bias[co];
    }
}

// initial conv [k0][k0][C][F] -> [K0 / 32][FP][32], k = tap C + c (hi; lo for split precision)
__global__ void pack_w0_kernel(const float* w, const float* scale, const float* bias, uint16_t* w0, uint16_t* w0lo,
                               float* b0, int KF, int F, int FP) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < KF; i += gridDim.x * blockDim.x) {
        const int k = i / F, co = i % F;
        const float v = f_mul(w[i], scale[co]);
        const size_t o = ((size_t)(k / 32) * FP + co) * 32 + (k % 32);
        w0[o] = f2bf(v);
        if (w0lo) w0lo[o] = lo_of_dev(v);
        if (k == 0) b0[co] = bias[co];
    }
}

// dst[i ds] = src[i ss] (mode 0), * sc[i] (1), * sc[0] (2)
struct VecJob {
    const float* src;
    float* dst;
    const float* sc;
    int n, ss, ds, mode;
};
__global__ void vec_kernel(const VecJob* jobs) {
    const VecJob j = jobs[blockIdx.x];
    for (int i = threadIdx.x; i < j.n; i += blockDim.x) {
        const float v = j.src[(size_t)i * j.ss];
        j.dst[(size_t)i * j.ds] = j.mode == 0 ? v : f_mul(v, j.mode == 1 ? j.sc[i] : j.sc[0]);
    }
}

// policy_gemm_kernel's A fragments of one role (the host path's pdp loop)
__global__ void pack_pdp_kernel(const float* pd, uint16_t* dst, int P, int K, int nkt, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int e = (int)(i % 8), l = (int)((i / 8) % 64);
        const size_t t = i / (8 * 64);      // jt * nkt + kt
        const int kt = (int)(t % nkt), jt = (int)(t / nkt);
        const int j = 16 * jt + (l & 15), k = 32 * kt + 8 * (l >> 4) + e;
        if (j >= P || k >= K) continue;
        const float v = pd[(size_t)k * P + j];
        const size_t o = ((t * 2) * 64 + l) * 8 + e;
        dst[o] = f2bf(v);
        dst[o + 64 * 8] = lo_of_dev(v);
    }
}
}  // namespace

extern "C" int gz_net_set_weights_device(gz_net* net, const float* d_blob, size_t count) {
    if (!net || !d_blob) return fail("null argument");
    if (count != net->nweights)
        return fail("weight count mismatch: got " + std::to_string(count) + " expected " + std::to_string(net->nweights));
    if (getenv("GZ_HOST_WEIGHT_ROLL")) {   // diagnostics: the round-trip path (D2H, host fold / pack, H2D)
        std::vector<float> h(count);
        HIPCHK(hipSetDevice(net->device));
        HIPCHK(hipMemcpy(h.data(), d_blob, count * 4, hipMemcpyDeviceToHost));
        return gz_net_set_weights(net, h.data(), count);
    }
    const gz_net_desc& d = net->d;
    const int F = d.cnn_filter_size, FP = net->fpad, B = d.residual_layers, R = d.role_count, S = d.se_units;
    const int HW = d.input_columns * d.input_rows, P2 = net->p2, NL = cal_layers(d);
    const int VH = d.value_hidden_size, VK = value_features(d);
    const BlobPlan P = blob_plan(d, d_blob);
    if (P.consumed != count) return fail("internal: blob plan mismatch");
    const ImageLayout I = image_layout(net);
    HIPCHK(hipSetDevice(net->device));
    // The blob's producer (an RCCL broadcast, a copy on torch's stream, ...) ran on some other
    // stream: net->stream is non-blocking, so nothing orders the fold / pack kernels after it.  Wait
    // for all work issued to the device so far (a roll is rare; the runner applies it between
    // launches, whose in-flight ones gz_net_set_weights waits for anyway).
    HIPCHK(hipDeviceSynchronize());
    hipStream_t st = net->stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    char* m = nullptr;
    float* fold = nullptr;
    void* jobs_d = nullptr;
    auto cleanup = [&]() {
        if (fold) (void)hipFree(fold);
        if (jobs_d) (void)hipFree(jobs_d);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    };
    auto bail = [&](const std::string& what, hipError_t e) {
        cleanup();
        if (m) (void)hipFree(m);
        return fail(what + ": " + hipGetErrorString(e));
    };
    hipError_t e;
    if ((e = hipMalloc((void**)&m, I.total)) != hipSuccess) return bail("hipMalloc image", e);
    if ((e = hipMalloc((void**)&fold, (size_t)std::max(P.fold_floats, 1) * 4)) != hipSuccess) return bail("hipMalloc fold", e);
    if ((e = hipMemsetAsync(m, 0, I.total, st)) != hipSuccess) return bail("hipMemsetAsync", e);

    // BN folds (every BNRef of the plan)
    std::vector<BNJob> bj;
    auto addbn = [&](const BNRef& b) { bj.push_back(BNJob{b.g, b.be, b.mu, b.var, b.cb, b.n, b.out}); };
    addbn(P.bn0);
    for (const BNRef& b : P.bnconv) addbn(b);
    for (const BNRef& b : P.pre) addbn(b);
    for (int r = 0; r < R; ++r) addbn(P.hbn[r]);
    for (const BNRef& b : P.clbn) addbn(b);
    if (NL == 0) addbn(P.vbn);
    // the small vectors derived from the folds (heads' 1x1 convs, per-layer value convs, v2 pre-BN)
    std::vector<VecJob> vj;
    auto sc_of = [&](const BNRef& b) { return fold + b.out; };
    auto bi_of = [&](const BNRef& b) { return fold + b.out + b.n; };
    char* const mc = m;
    float* wh = (float*)(mc + I.wh);
    float* bh = (float*)(mc + I.bh);
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < 2; ++c) {
            vj.push_back(VecJob{P.hw[r] + c, wh + (size_t)(2 * r + c) * FP, sc_of(P.hbn[r]) + c, F, 2, 1, 2});
            vj.push_back(VecJob{bi_of(P.hbn[r]) + c, bh + 2 * r + c, nullptr, 1, 1, 1, 0});
        }
    for (int j = 0; j < NL; ++j) {
        vj.push_back(VecJob{P.clw[j], (float*)(mc + I.wcl) + (size_t)j * FP, sc_of(P.clbn[j]), F, 1, 1, 2});
        vj.push_back(VecJob{bi_of(P.clbn[j]), (float*)(mc + I.bcl) + j, nullptr, 1, 1, 1, 0});
    }
    if (NL == 0) {
        vj.push_back(VecJob{P.vw, wh + (size_t)(2 * R) * FP, sc_of(P.vbn), F, 1, 1, 2});
        vj.push_back(VecJob{bi_of(P.vbn), bh + 2 * R, nullptr, 1, 1, 1, 0});
    }
    for (int blk = 0; blk < (int)P.pre.size(); ++blk) {
        vj.push_back(VecJob{sc_of(P.pre[blk]), (float*)(mc + I.pre) + (size_t)(2 * blk) * FP, nullptr, F, 1, 1, 0});
        vj.push_back(VecJob{bi_of(P.pre[blk]), (float*)(mc + I.pre) + (size_t)(2 * blk + 1) * FP, nullptr, F, 1, 1, 0});
    }
    const size_t bj_bytes = bj.size() * sizeof(BNJob), vj_bytes = vj.size() * sizeof(VecJob);
    if ((e = hipMalloc(&jobs_d, bj_bytes + vj_bytes + 16)) != hipSuccess) return bail("hipMalloc jobs", e);
    BNJob* bj_d = (BNJob*)jobs_d;
    VecJob* vj_d = (VecJob*)((char*)jobs_d + ((bj_bytes + 15) & ~(size_t)15));
    if ((e = hipMemcpyAsync(bj_d, bj.data(), bj_bytes, hipMemcpyHostToDevice, st)) != hipSuccess) return bail("jobs", e);
    if (!vj.empty() && (e = hipMemcpyAsync(vj_d, vj.data(), vj_bytes, hipMemcpyHostToDevice, st)) != hipSuccess)
        return bail("jobs", e);
    hipLaunchKernelGGL(bn_fold_kernel, dim3((unsigned)bj.size()), dim3(256), 0, st, bj_d, fold);
    {   // initial conv
        const int KF = initial_kernel(d) * initial_kernel(d) * d.input_channels * F;
        hipLaunchKernelGGL(pack_w0_kernel, dim3((KF + 255) / 256), dim3(256), 0, st, P.w0, sc_of(P.bn0), bi_of(P.bn0),
                           (uint16_t*)(mc + I.w0), P2 == 2 ? (uint16_t*)(mc + I.w0lo) : (uint16_t*)nullptr,
                           (float*)(mc + I.b0), KF, F, FP);
    }
    for (int c = 0; c < 2 * B; ++c) {
        const size_t n = (size_t)9 * F * F;
        hipLaunchKernelGGL(pack_conv_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                           P.wconv[c], sc_of(P.bnconv[c]), bi_of(P.bnconv[c]),
                           (uint16_t*)(mc + I.wres) + (size_t)P2 * c * 9 * FP * FP, (float*)(mc + I.bres) + (size_t)c * FP,
                           F, FP, P2);
    }
    if (!vj.empty()) hipLaunchKernelGGL(vec_kernel, dim3((unsigned)vj.size()), dim3(256), 0, st, vj_d);
    // plain copies: the dense heads (output dimension padded to 4), biases, squeeze-excite layers
    auto cp = [&](void* dst, const void* src, size_t bytes) { return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st); };
    auto cp2 = [&](void* dst, size_t dpitch, const void* src, size_t spitch, size_t w, size_t h) {
        return hipMemcpy2DAsync(dst, dpitch, src, spitch, w, h, hipMemcpyDeviceToDevice, st);
    };
    for (int r = 0; r < R; ++r) {
        const int Pr = d.policy_dist_count[r];
        if ((e = cp2(mc + I.pd[r], (size_t)((Pr + 3) & ~3) * 4, P.pd[r], (size_t)Pr * 4, (size_t)Pr * 4, (size_t)2 * HW)) != hipSuccess)
            return bail("policy dense", e);
        if ((e = cp(mc + I.pb[r], P.pb[r], (size_t)Pr * 4)) != hipSuccess) return bail("policy bias", e);
    }
    if ((e = cp2(mc + I.vhw, (size_t)((VH + 3) & ~3) * 4, P.vhw, (size_t)VH * 4, (size_t)VH * 4, (size_t)VK)) != hipSuccess)
        return bail("value dense", e);
    if ((e = cp(mc + I.vhb, P.vhb, (size_t)VH * 4)) != hipSuccess) return bail("value bias", e);
    if ((e = cp(mc + I.vdw, P.vdw, (size_t)VH * d.num_values * 4)) != hipSuccess) return bail("value out", e);
    if ((e = cp(mc + I.vdb, P.vdb, (size_t)d.num_values * 4)) != hipSuccess) return bail("value out bias", e);
    for (int blk = 0; blk < (int)P.se_c.size(); ++blk) {
        if ((e = cp((float*)(mc + I.sew1) + (size_t)blk * FP * S, P.se_c[blk], (size_t)F * S * 4)) != hipSuccess)
            return bail("squeeze-excite", e);
        if ((e = cp2((float*)(mc + I.sew2) + (size_t)blk * S * FP, (size_t)FP * 4, P.se_g[blk], (size_t)F * 4, (size_t)F * 4,
                     (size_t)S)) != hipSuccess)
            return bail("squeeze-excite", e);
    }
    if (net->gemm_heads) {
        const int K = 2 * HW, nkt = (K + 31) / 32;
        for (int r = 0; r < R; ++r) {
            const size_t n = I.n_pdp[r] / 2;   // (hi, lo) pairs
            hipLaunchKernelGGL(pack_pdp_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                               P.pd[r], (uint16_t*)(mc + I.pdp[r]), d.policy_dist_count[r], K, nkt, n);
        }
    }
    if ((e = hipGetLastError()) != hipSuccess) return bail("pack kernels", e);
    if ((e = hipEventRecord(e1, st)) != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess) return bail("roll sync", e);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    net->last_roll_ms = ms;
    cleanup();
    return install_image(net, m, I);
}

extern "C" double gz_net_last_roll_ms(const gz_net* net) { return net ? (double)net->last_roll_ms : -1.0; }

// diagnostics: the device weight image (out == NULL: its size)
extern "C" size_t gz_net_copy_weight_image(gz_net* net, void* out, size_t cap) {
    if (!net || !net->dmem) return 0;
    std::lock_guard<std::mutex> wl(net->wmu);
    if (!out) return net->image_bytes;
    const size_t n = std::min(cap, net->image_bytes);
    if (hipSetDevice(net->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, net->dmem, n, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return n;
}

static int launch_segments(gz_net* net, hipStream_t stream, const gz_segment* segs, int nseg,
                           hipEvent_t mid = nullptr) {
    if (nseg < 1 || nseg > kMaxSegments) return fail("segment count out of range (1.." + std::to_string(kMaxSegments) + ")");
    // the weight image stays valid until this launch is queued (gz_net_set_weights frees a replaced
    // image only after a device sync)
    std::lock_guard<std::mutex> wl(net->wmu);
    if (!net->has_weights) return fail("weights not set");
    KParams kp = net->kp;
    int n = 0;
    for (int i = 0; i < nseg; ++i) {
        if (segs[i].rows < 0) return fail("negative segment rows");
        Segment& g = kp.seg[i];
        g.row0 = n;
        g.planes = segs[i].planes;
        for (int r = 0; r < kp.R; ++r) g.pol[r] = segs[i].policies[r];
        g.val = segs[i].values;
        n += segs[i].rows;
    }
    if (n <= 0) return 0;
    kp.n = n;
    kp.nseg = nseg;
    kp.stamps = net->stamps_on ? net->d_stamps : nullptr;
    {   // head-feature scratch of this stream (grown with a device sync: rare, sizes only increase)
        std::lock_guard<std::mutex> lk(net->feat_mu);
        auto& f = net->feat[stream];
        if (f.second < n) {
            if (f.first) {
                HIPCHK(hipDeviceSynchronize());
                HIPCHK(hipFree(f.first));
                f.first = nullptr;
            }
            const int cap = std::max(n, 8192);
            HIPCHK(hipMalloc((void**)&f.first, (size_t)cap * kp.FS * sizeof(float)));
            f.second = cap;
        }
        kp.feat = f.first;
        kp.glog = nullptr;
        if (net->gemm_heads) {
            auto& g = net->glog[stream];
            if (g.second < n) {
                if (g.first) {
                    HIPCHK(hipDeviceSynchronize());
                    HIPCHK(hipFree(g.first));
                    g.first = nullptr;
                }
                const int cap = std::max(n, 8192);
                HIPCHK(hipMalloc((void**)&g.first, (size_t)cap * kp.plog * sizeof(float)));
                g.second = cap;
            }
            kp.glog = g.first;
        }
    }
    const gz_net::Trunk& t = n >= net->large_min_rows ? net->large : net->small;
    kp.resid = nullptr;
    if (t.resid_bytes) {
        std::lock_guard<std::mutex> lk(net->feat_mu);
        auto& f = net->resid[stream];
        const size_t need = (size_t)((n + t.nb - 1) / t.nb) * t.resid_bytes;
        if (f.second < need) {
            if (f.first) {
                HIPCHK(hipDeviceSynchronize());
                HIPCHK(hipFree(f.first));
                f.first = nullptr;
            }
            const size_t cap = std::max(need, (size_t)1024 * t.resid_bytes);
            HIPCHK(hipMalloc((void**)&f.first, cap));
            f.second = cap;
        }
        kp.resid = (f32x4*)f.first;
    }
    kp.btab_off = t.btab_off;
    kp.se_off = t.se_off;
    kp.cal_off = t.cal_off;
    void* args[] = {&kp};
    HIPCHK(hipLaunchKernel(t.fn, dim3((n + t.nb - 1) / t.nb), dim3(t.threads), args, t.smem, stream));
    if (mid) HIPCHK(hipEventRecord(mid, stream));
    if (net->gemm_heads) {
        int maxjt = 0;
        for (int r = 0; r < kp.R; ++r) maxjt = std::max(maxjt, (kp.P[r] + 15) / 16);
        HIPCHK(hipLaunchKernel((const void*)&policy_gemm_kernel, dim3((n + 63) / 64, (maxjt + 7) / 8, kp.R), dim3(256),
                               args, 0, stream));
    }
    if (!t.fused_heads)
        HIPCHK(hipLaunchKernel((const void*)&heads_kernel, dim3((n + kHeadBoards - 1) / kHeadBoards), dim3(256), args,
                               net->heads_smem, stream));
    return 0;
}

static int launch(gz_net* net, hipStream_t stream, const float* d_planes, int n,
                  float* const* d_pol, float* d_val) {
    gz_segment sg{};
    sg.rows = n;
    sg.planes = d_planes;
    for (int r = 0; r < net->kp.R; ++r) sg.policies[r] = d_pol[r];
    sg.values = d_val;
    return launch_segments(net, stream, &sg, 1);
}

extern "C" int gz_net_forward_device(gz_net* net, void* stream, const float* d_planes, int n,
                                     float* const* d_policies, float* d_values) {
    if (!net) return fail("null net");
    return launch(net, (hipStream_t)stream, d_planes, n, d_policies, d_values);
}

extern "C" int gz_net_forward_segments(gz_net* net, void* stream, const gz_segment* segs, int nseg) {
    if (!net || !segs) return fail("null argument");
    return launch_segments(net, (hipStream_t)stream, segs, nseg);
}

extern "C" int gz_net_forward_segments_ev(gz_net* net, void* stream, const gz_segment* segs, int nseg,
                                          void* trunk_done_event) {
    if (!net || !segs) return fail("null argument");
    return launch_segments(net, (hipStream_t)stream, segs, nseg, (hipEvent_t)trunk_done_event);
}

extern "C" int gz_net_forward(gz_net* net, const float* planes, int n, float* const* policies, float* values) {
    if (!net || !planes || !policies || !values) return fail("null argument");
    if (n <= 0) return 0;
    const gz_net_desc& d = net->d;
    const size_t in_f = (size_t)d.input_channels * d.input_columns * d.input_rows;
    size_t out_f = d.num_values;
    for (int r = 0; r < d.role_count; ++r) out_f += d.policy_dist_count[r];
    HIPCHK(hipSetDevice(net->device));
    if (n > net->io_cap) {
        if (net->d_io) HIPCHK(hipFree(net->d_io));
        net->d_io = nullptr;
        HIPCHK(hipMalloc((void**)&net->d_io, (size_t)n * (in_f + out_f) * 4 + 1024));
        net->io_cap = n;
    }
    float* d_in = net->d_io;
    float* d_pol[GZ_MAX_ROLES];
    float* p = d_in + (size_t)n * in_f;
    for (int r = 0; r < d.role_count; ++r) { d_pol[r] = p; p += (size_t)n * d.policy_dist_count[r]; }
    float* d_val = p;
    HIPCHK(hipMemcpyAsync(d_in, planes, (size_t)n * in_f * 4, hipMemcpyHostToDevice, net->stream));
    const bool stamps = getenv("GZ_KERNEL_STAMPS") != nullptr;
    const int grid = n;   // >= workgroups of either trunk variant
    if (stamps && grid > net->stamp_cap) {
        if (net->d_stamps) HIPCHK(hipFree(net->d_stamps));
        HIPCHK(hipMalloc((void**)&net->d_stamps, (size_t)grid * 8 * sizeof(unsigned long long)));
        net->stamp_cap = grid;
    }
    if (stamps) HIPCHK(hipMemsetAsync(net->d_stamps, 0, (size_t)grid * 8 * sizeof(unsigned long long), net->stream));
    HIPCHK(hipEventRecord(net->ev0, net->stream));
    net->stamps_on = stamps;
    const int lrc = launch(net, net->stream, d_in, n, d_pol, d_val);
    net->stamps_on = false;
    if (lrc) return -1;
    HIPCHK(hipEventRecord(net->ev1, net->stream));
    for (int r = 0; r < d.role_count; ++r)
        HIPCHK(hipMemcpyAsync(policies[r], d_pol[r], (size_t)n * d.policy_dist_count[r] * 4, hipMemcpyDeviceToHost, net->stream));
    HIPCHK(hipMemcpyAsync(values, d_val, (size_t)n * d.num_values * 4, hipMemcpyDeviceToHost, net->stream));
    HIPCHK(hipStreamSynchronize(net->stream));
    HIPCHK(hipEventElapsedTime(&net->last_ms, net->ev0, net->ev1));
    if (stamps) {
        std::vector<unsigned long long> h((size_t)grid * 8);
        HIPCHK(hipMemcpy(h.data(), net->d_stamps, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        // the launch ran ceil(n / NB) workgroups: average over the ones that stamped
        for (int i = 0; i < 8; ++i) net->stamp_avg[i] = 0;
        int wgs = 0;
        for (int b = 0; b < grid; ++b) {
            if (h[(size_t)b * 8] == 0 || h[(size_t)b * 8 + 4] == 0) continue;
            ++wgs;
            for (int i = 1; i < 5; ++i) net->stamp_avg[i] += (double)(h[(size_t)b * 8 + i] - h[(size_t)b * 8 + i - 1]);
        }
        for (int i = 1; i < 5; ++i) net->stamp_avg[i] = wgs ? net->stamp_avg[i] / wgs : 0.0;
        net->stamp_avg[0] = wgs;
    }
    return 0;
}

extern "C" int gz_net_stamp_avg(const gz_net* net, double* out8) {
    for (int i = 0; i < 8; ++i) out8[i] = net->stamp_avg[i];
    return 0;
}

extern "C" float gz_net_last_kernel_ms(const gz_net* net) { return net ? net->last_ms : 0.f; }

extern "C" int gz_net_set_output_logits(gz_net* net, int on) {
    if (!net) return fail("null net");
    std::lock_guard<std::mutex> wl(net->wmu);
    net->kp.logits = on ? 1 : 0;
    return 0;
}

extern "C" int gz_net_large_min_rows(const gz_net* net) { return net ? net->large_min_rows : 0; }

extern "C" const char* gz_net_kernel_name(const gz_net* net, int large) {
    if (!net) return "";
    return (large ? net->large : net->small).name.c_str();
}

extern "C" int gz_net_wave_rows(const gz_net* net) {
    if (!net) return 0;
    return (net->large_min_rows < (1 << 30) ? net->large.nb : net->small.nb) * kCUs;
}
