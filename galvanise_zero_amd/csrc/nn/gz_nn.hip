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
// selectable (GZ_KERNEL_VARIANT=24), bit-identical.  kLargeFallback: where kLargeVariant is not
// compiled for a geometry.
constexpr int kSmallVariant = 11, kLargeVariant = 21, kLargeFallback = 21, kLargeMinRows = 257;
constexpr int kCUs = 256;

static KernelChoice select_kernel(int fpad, int pt, int v, int precision, bool v2) {
    if (pt < 1 || pt > kMaxPT) return KernelChoice{};
    return trunk_variant(fpad, pt, v, precision, v2);
}

// ---- bf16 (round to nearest even) -------------------------------------------------------------
static inline uint16_t f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
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
    const int fpad = padded_filters(d.cnn_filter_size);
    const int npos_ = d.input_columns * d.input_rows;
    const int pt = (npos_ + 15) / 16;
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
    if (kl.fn && !wg_fits(kl)) kl = KernelChoice{};
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
    // trunk conv `conv` [3][3][F][F] * scale[co] -> [tap][kc][co][32] (split precision:
    // [tap][kc][co][hi 32 | lo 32]), bias[co] -> bres
    auto pack_conv = [&](int conv, const float* w, const std::vector<float>& scale, const std::vector<float>& bias) {
        uint16_t* dst = wres.data() + (size_t)P2 * conv * 9 * FP * FP;
        for (int co = 0; co < F; ++co) {
            bres[(size_t)conv * FP + co] = bias[co];
            for (int tap = 0; tap < 9; ++tap)
                for (int ci = 0; ci < F; ++ci) {
                    const float v = w[((size_t)tap * F + ci) * F + co] * scale[co];
                    const size_t o = ((((size_t)tap * KC + ci / 32) * FP + co) * P2) * 32 + (ci % 32);
                    dst[o] = f2bf(v);
                    if (P2 == 2) dst[o + 32] = lo_of(v);
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

    // device layout
    Layout L;
    const size_t o_w0 = L.alloc(w0.size() * 2), o_w0lo = L.alloc(std::max<size_t>(w0lo.size(), 1) * 2);
    const size_t o_b0 = L.alloc(b0.size() * 4);
    const size_t o_wres = L.alloc(wres.size() * 2), o_bres = L.alloc(bres.size() * 4);
    const size_t o_wh = L.alloc(wh.size() * 4), o_bh = L.alloc(bh.size() * 4);
    const size_t o_wcl = L.alloc(wcl.size() * 4), o_bcl = L.alloc(bcl.size() * 4);
    size_t o_pd[GZ_MAX_ROLES], o_pb[GZ_MAX_ROLES];
    for (int r = 0; r < R; ++r) {
        o_pd[r] = L.alloc(pdq[r].size() * 4);
        o_pb[r] = L.alloc((size_t)d.policy_dist_count[r] * 4);
    }
    const size_t o_vhw = L.alloc(vhq.size() * 4), o_vhb = L.alloc(d.value_hidden_size * 4);
    const size_t o_pre = L.alloc(pre.size() * 4), o_sew1 = L.alloc(sew1.size() * 4), o_sew2 = L.alloc(sew2.size() * 4);
    const size_t o_vdw = L.alloc((size_t)d.value_hidden_size * d.num_values * 4), o_vdb = L.alloc(d.num_values * 4);
    // policy_gemm_kernel's A fragments: W^T tiles [jt][kt][hi | lo][64 lanes][8 k] bf16, lane l holding
    // row j = 16 jt + l % 16 and k = 32 kt + 8 (l / 16) + e (zero padded)
    std::vector<std::vector<uint16_t>> pdp(R);
    size_t o_pdp[GZ_MAX_ROLES] = {};
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
            o_pdp[r] = L.alloc(pdp[r].size() * 2);
        }
    }

    std::vector<char> img(L.off, 0);
    auto put = [&](size_t off, const void* src, size_t bytes) { std::memcpy(img.data() + off, src, bytes); };
    put(o_w0, w0.data(), w0.size() * 2);
    if (P2 == 2) put(o_w0lo, w0lo.data(), w0lo.size() * 2);
    put(o_b0, b0.data(), b0.size() * 4);
    put(o_wres, wres.data(), wres.size() * 2);
    put(o_bres, bres.data(), bres.size() * 4);
    put(o_wh, wh.data(), wh.size() * 4);
    put(o_bh, bh.data(), bh.size() * 4);
    put(o_wcl, wcl.data(), wcl.size() * 4);
    put(o_bcl, bcl.data(), bcl.size() * 4);
    for (int r = 0; r < R; ++r) {
        put(o_pd[r], pdq[r].data(), pdq[r].size() * 4);   // Keras [2HW][P_r] (k-major), rows padded to P4
        put(o_pb[r], pbias[r], (size_t)d.policy_dist_count[r] * 4);
    }
    put(o_vhw, vhq.data(), vhq.size() * 4);   // Keras [VK][VH], rows padded to VH4
    put(o_pre, pre.data(), pre.size() * 4);
    put(o_sew1, sew1.data(), sew1.size() * 4);
    put(o_sew2, sew2.data(), sew2.size() * 4);
    put(o_vhb, vhb, d.value_hidden_size * 4);
    put(o_vdw, vdw, (size_t)d.value_hidden_size * d.num_values * 4);
    put(o_vdb, vdb, d.num_values * 4);
    if (net->gemm_heads)
        for (int r = 0; r < R; ++r) put(o_pdp[r], pdp[r].data(), pdp[r].size() * 2);

    HIPCHK(hipSetDevice(net->device));
    char* m = nullptr;
    HIPCHK(hipMalloc((void**)&m, L.off));
    if (hipMemcpy(m, img.data(), L.off, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(m);
        return fail("weight upload failed");
    }
    // swap under the lock launch_segments takes: a launcher thread running a generation roll sees
    // either the old or the new image, never a mix
    std::unique_lock<std::mutex> wl(net->wmu);
    char* old = net->dmem;
    net->dmem = m;
    KParams& kp = net->kp;
    kp.w0 = (const __bf16*)(m + o_w0);
    kp.w0lo = (const __bf16*)(m + o_w0lo);
    kp.b0 = (const float*)(m + o_b0);
    kp.wres = (const __bf16*)(m + o_wres);
    kp.bres = (const float*)(m + o_bres);
    kp.wh = (const float*)(m + o_wh);
    kp.bh = (const float*)(m + o_bh);
    kp.wcl = (const float*)(m + o_wcl);
    kp.bcl = (const float*)(m + o_bcl);
    for (int r = 0; r < R; ++r) {
        kp.pd[r] = (const float*)(m + o_pd[r]);
        kp.pb[r] = (const float*)(m + o_pb[r]);
    }
    kp.vhw = (const float*)(m + o_vhw);
    kp.vhb = (const float*)(m + o_vhb);
    kp.vdw = (const float*)(m + o_vdw);
    kp.vdb = (const float*)(m + o_vdb);
    kp.pre = (const float*)(m + o_pre);
    kp.sew1 = (const float*)(m + o_sew1);
    kp.sew2 = (const float*)(m + o_sew2);
    for (int r = 0; r < R; ++r) kp.pdp[r] = net->gemm_heads ? (const __bf16*)(m + o_pdp[r]) : nullptr;
    net->has_weights = true;
    wl.unlock();
    if (old) {   // launches already queued may still read the old image
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipFree(old));
    }
    return 0;
}

extern "C" int gz_net_set_weights_device(gz_net* net, const float* d_blob, size_t count) {
    if (!net || !d_blob) return fail("null argument");
    std::vector<float> h(count);
    HIPCHK(hipSetDevice(net->device));
    HIPCHK(hipMemcpy(h.data(), d_blob, count * 4, hipMemcpyDeviceToHost));
    return gz_net_set_weights(net, h.data(), count);
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
