/* gzero_nn.h -- C-ABI of the MI355X policy/value network forward (libgz_nn.so).
 *
 * Replaces, for the self-play hot path, the Keras model the reference runs through
 *   NeuralNetwork.get_model().predict_on_batch(X)      src/ggpzero/util/cppinterface.py:119
 * built by get_network_model()                          src/ggpzero/nn/model.py:154-296 (v1 path)
 * and loaded by Manager.load_network / create_new_network   src/ggpzero/nn/manager.py:96-139.
 *
 * All entry points take plain pointers and sizes.  Every function returning int returns 0 on
 * success and a negative code on failure; gz_nn_last_error() then holds a message (thread-local).
 */
#ifndef GZERO_NN_H
#define GZERO_NN_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GZ_MAX_ROLES 4

/* Mirror of the forward-relevant fields of confs.NNModelConfig (src/ggpzero/defs/confs.py:127-151)
 * plus GenerationDescription.draw_head (num_values 3) and the Flatten data_format of the model
 * file. */
typedef struct gz_net_desc {
    int input_channels;                       /* C                                  */
    int input_columns;                        /* H = len(y_cords)  (bases.py:115)   */
    int input_rows;                           /* W = len(x_cords)  (bases.py:111)   */
    int cnn_filter_size;                      /* F                                  */
    int cnn_kernel_size;                      /* must be 3                          */
    int residual_layers;                      /* B                                  */
    int role_count;                           /* R = number of policy heads         */
    int policy_dist_count[GZ_MAX_ROLES];      /* P_r                                */
    int value_hidden_size;
    int num_values;                           /* 2, or 3 with a draw head           */
    int leaky_relu;                           /* 0: relu, 1: LeakyReLU(alpha=0.03)  */
    int flatten_nchw;                         /* 0: Keras>=2.1.6 (H,W,C) flatten; 1: legacy (C,H,W) */
    /* legacy v1 model files (data/breakthrough/models/x6_102.json, keras 2.1.3): */
    int conv_bias;                            /* every Conv2D has use_bias: a bias after each kernel */
    int value_bn;                             /* BatchNormalization after the value head's 1x1 conv  */
    int value_sigmoid;                        /* value Dense activation sigmoid (else softmax)      */
    /* Arithmetic of the residual trunk (build extension; the reference runs fp32 TF kernels):
     *   GZ_PRECISION_BF16 (0 or 1): bf16 operands, fp32 accumulation and residual stream;
     *   GZ_PRECISION_SPLIT (3): each fp32 operand as bf16 hi + bf16 lo and each product as
     *   hi*hi + hi*lo + lo*hi on the MFMA (~16 significant bits per operand against fp32's 24, fp32
     *   accumulation: pre-softmax logits within ~1e-4 relative of an fp32 forward, the per-config
     *   bounds of nn/tolerance.py); F <= 128 on boards <= 64 positions two per workgroup, larger
     *   boards (up to 19 x 19) one per workgroup, by two passes per conv where the hi + lo image
     *   exceeds the LDS (F = 256 on 13 x 13, F = 128 on 19 x 19).  The heads' 1x1 convs, softmaxes and value MLP are
     *   fp32 in both modes; the policy Dense is fp32 except for single-image nets with a policy of
     *   >= 512 moves (amazons), whose policy Dense of the whole launch runs as one bf16x3 split MFMA
     *   GEMM in both modes (policy_gemm_kernel; GZ_NO_GEMM_HEADS=1 keeps it fp32 on the VALU).
     *   Stated error per config: galvanise_zero_amd/nn/tolerance.py. */
    int precision;
    /* v2 (pre-activation) trunk, model.py:78-151 (the reference's features=True templates and its
     * non-legacy model files); all zero = v1. */
    int resnet_v2;                            /* blocks BN-act-conv-BN-act-conv [SE], add, no act    */
    int initial_kernel;                       /* 1 or 3; 0 = model.py's (1 for v2, 3 for v1)        */
    int initial_bn;                           /* v2: BN + act after the initial conv (0: bare conv)  */
    int se_units;                             /* squeeze-excite compress units, 0 = none (<= 64)     */
    int global_pooling_value;                 /* value features = [trunk channel means (F), conv (HW)] */
    /* v2 only, model.py:251-260: the value head reads every trunk layer (the initial conv block's
     * output and each residual block's add), each through its own 1x1 conv + BN + act: (B + 1) HW
     * features in layer order.  Such nets run the dense heads in a separate heads launch. */
    int concat_all_layers;
} gz_net_desc;

#define GZ_PRECISION_BF16 1
#define GZ_PRECISION_SPLIT 3

typedef struct gz_net gz_net;

/* Create a network on HIP device `device`.  Returns NULL on error (see gz_nn_last_error). */
gz_net* gz_net_create(const gz_net_desc* desc, int device);
void gz_net_destroy(gz_net* net);

/* Number of float32 values of the canonical weight blob (layout: galvanise_zero_amd/nn/desc.py
 * weight_spec(): Keras storage order, conv HWIO, BN as gamma,beta,mean,var, dense [in][out]). */
size_t gz_net_weight_count(const gz_net* net);

/* Upload weights from a host float32 blob (BN folded + packed to bf16 on the host).  Safe while a
 * runner is launching on this net (generation roll): launches issued after the call use the new
 * weights, launches already in flight finish on the old ones, which are freed after a device sync. */
int gz_net_set_weights(gz_net* net, const float* blob, size_t count);

/* Upload weights from a *device* float32 blob (e.g. after an RCCL broadcast into device memory): the
 * BN fold and the bf16 (hi / lo) packing run as HIP kernels reading the blob in place -- no PCIe
 * round trip -- and produce the byte-identical image gz_net_set_weights builds on the host.  The
 * generation roll of a live runner (gz_runner_update_network with device_blob = 1) takes this path.
 * The blob may still be in flight on any stream (a broadcast, an async copy): the call first waits
 * for all work issued to the device (hipDeviceSynchronize), so no caller-side synchronisation is
 * needed. */
int gz_net_set_weights_device(gz_net* net, const float* d_blob, size_t count);
/* device milliseconds of the last gz_net_set_weights_device (fold + pack kernels and copies) */
double gz_net_last_roll_ms(const gz_net* net);
/* diagnostics: copies the packed device weight image to host memory (out == NULL: returns its size) */
size_t gz_net_copy_weight_image(gz_net* net, void* out, size_t cap);

/* One contiguous run of boards of a segmented launch.  Pointers may be device memory or pinned host
 * memory (hipHostMalloc): the kernel gathers planes from, and scatters outputs to, each segment
 * directly.  (The native runner DMAs each launch's planes to an HBM staging buffer on a copy stream
 * first and passes that as the planes; outputs go straight to the pools' pinned buffers.) */
#define GZ_MAX_SEGMENTS 32
typedef struct gz_segment {
    int rows;
    const float* planes;                      /* [rows][C][H][W] */
    float* policies[GZ_MAX_ROLES];            /* [rows][P_r] */
    float* values;                            /* [rows][num_values] */
} gz_segment;

/* Asynchronous forward of up to GZ_MAX_SEGMENTS segments on `stream`.  Nets whose trunk kernel
 * holds two activation images (F <= 128, and F = 256 up to 8 x 8) run the whole forward -- trunk and
 * dense heads -- in one launch (gz_net_heads_fused); single-image nets (F = 256 on 10 x 10 / 13 x 13)
 * launch the trunk (planes -> head features), then the policy GEMM for large policies, then the
 * heads kernel. */
int gz_net_forward_segments(gz_net* net, void* stream, const gz_segment* segs, int nseg);
/* Same, recording `trunk_done_event` (a hipEvent_t, may be NULL) after the trunk launch so the
 * caller can time the trunk kernel alone. */
int gz_net_forward_segments_ev(gz_net* net, void* stream, const gz_segment* segs, int nseg,
                               void* trunk_done_event);

/* Synchronous forward, host buffers: planes float32 [n][C][H][W] (the poll() buffer layout,
 * cppinterface.py:114); policies[r] float32 [n][P_r]; values float32 [n][num_values].
 * Equivalent of predict_on_batch on one batch. */
int gz_net_forward(gz_net* net, const float* planes, int n,
                   float* const* policies, float* values);

/* Asynchronous forward on a caller stream (hipStream_t passed as void*), device buffers. */
int gz_net_forward_device(gz_net* net, void* stream, const float* d_planes, int n,
                          float* const* d_policies, float* d_values);

/* Diagnostics: on != 0 makes later forwards write the heads' pre-activation outputs (policy logits
 * before the softmax, value logits before the softmax / sigmoid) instead of probabilities, so parity
 * tests can compare nets whose softmaxes saturate. */
int gz_net_set_output_logits(gz_net* net, int on);

/* Device time (ms) of the last gz_net_forward (both launches), measured with HIP events on its stream. */
float gz_net_last_kernel_ms(const gz_net* net);

/* Launches of at least this many rows run the two-boards-per-workgroup trunk variant, smaller ones
 * the one-board variant (both compute every row identically). */
int gz_net_large_min_rows(const gz_net* net);

/* The trunk kernel of launches below (large = 0) / from (large = 1) gz_net_large_min_rows rows, as
 * rocprofv3 names it (diagnostics: the bench reports its roofline per kernel). */
const char* gz_net_kernel_name(const gz_net* net, int large);

/* Rows one full wave of workgroups of the large variant covers (boards per workgroup x 256 CUs,
 * one trunk workgroup per CU): the native runner launches multiples of it beyond one wave. */
int gz_net_wave_rows(const gz_net* net);

/* Algorithmic FLOPs of one leaf evaluation (2 FLOP/MAC). */
double gz_net_flops_per_eval(const gz_net* net);

/* 1 when the large (two-board) trunk variant runs the dense policy / value heads itself (two-image
 * kernels: no separate heads launch), 0 when a separate heads kernel follows it. */
int gz_net_heads_fused(const gz_net* net);

const char* gz_nn_last_error(void);

/* Diagnostics: with GZ_KERNEL_STAMPS set in the environment, gz_net_forward records per-workgroup
 * s_memtime stamps at phase boundaries; out8[0] = workgroups averaged, out8[1..4] = their mean
 * cycles of (input + initial conv, residual trunk, head 1x1 convs + features, fused dense heads)
 * in the last call. */
int gz_net_stamp_avg(const gz_net* net, double* out8);

/* ---- native self-play driver (runner.hip) ----------------------------------------------------
 * Replaces the Python poll loop of the reference (cppinterface.py:131-144 driven by
 * distributed/worker.py:191) and its worker threads (supervisor.cpp:79-99,196-245) for the
 * steady state: num_threads engine threads x pools_per_thread game pools x batch_size games; one
 * launcher thread merges the pools waiting for predictions into segmented launches
 * (gz_net_forward_segments) that read planes from / write predictions to the pools' pinned host
 * buffers directly.
 * Uses the engine C-ABI (include/gzero_engine.h) for the pools. */
struct gz_sm;
struct gz_transformer;
struct gz_selfplay_config;
typedef struct gz_runner gz_runner;

typedef struct gz_runner_config {
    int device;
    int num_threads;
    int pools_per_thread;
    int batch_size;              /* games per pool = rows per NN batch */
    unsigned long long seed;
    long game_index_base;        /* global index of the first game (multi-GPU sharding) */
    int per_pool_unique_states;  /* 1: each pool owns its duplicate filter (deterministic per pool);
                                    0: one filter shared by every pool (reference, supervisor.cpp:31) */
    int keep_samples;            /* 1: queue samples for gz_runner_fetch_samples; 0: count and drop */
    int max_launch_rows;         /* cap on rows merged into one launch (0: no cap beyond 32 pools) */
    int min_launch_rows;         /* hold a launch until this many rows are queued ... (0: launch at once) */
    int max_launch_wait_us;      /* ... or its oldest pool has waited this long */
} gz_runner_config;

typedef struct gz_runner_stats {
    long batches;                /* NN forwards completed */
    long rows;                   /* leaf evaluations completed */
    double kernel_ms;            /* summed forward device time (HIP events around trunk + heads launches) */
    double trunk_ms;             /* summed trunk-kernel device time (events around the trunk launch) */
    long kernel_launches;
    long games_completed;
    long games_with_samples;
    long samples;
    long no_samples;
    long resigns;
    long aborts;
    long dupes;
    long segments;               /* pools merged into launches, summed over launches */
    long completed_game_evals;   /* NN evaluations consumed by the completed games */
    long large_launches;         /* launches that ran the two-boards-per-workgroup trunk variant */
    long large_rows;
    double large_trunk_ms;
    double engine_idle_ms;       /* summed over engine threads: time with none of the thread's pools ready */
    long tree_playouts;          /* tree playouts of all games (NN-free ones = tree_playouts - rows) */
    long large_rounds;           /* workgroup rounds of the large launches: sum of ceil(rows / gz_net_wave_rows) */
    long split_launches;         /* launches holding part of a pool's batch (exact-round composition) */
} gz_runner_stats;

gz_runner* gz_runner_create(gz_net* net, const struct gz_sm* sm, const struct gz_transformer* t,
                            const gz_runner_config* cfg, const struct gz_selfplay_config* conf,
                            const int* policy_sizes, int num_policies, int num_values);
int gz_runner_start(gz_runner* r);   /* once per runner: a stopped runner cannot be restarted */
int gz_runner_wait_batches(gz_runner* r, long total_batches, double timeout_s);
int gz_runner_wait_rows(gz_runner* r, long total_rows, double timeout_s);
int gz_runner_stats_get(gz_runner* r, gz_runner_stats* out);
int gz_runner_stop(gz_runner* r);
void gz_runner_destroy(gz_runner* r);
/* Samples queued since the last call, as one JSON array of datadesc.Sample records
 * (supervisor_impl.cpp:75-118 field names), or NULL when none; free with gz_free. */
char* gz_runner_fetch_samples(gz_runner* r);
/* clear_unique_states (supervisor_impl.cpp:138-144) at a generation roll (worker.py:160); safe while
 * the runner is running. */
int gz_runner_clear_unique_states(gz_runner* r);
/* Generation roll on a live runner (worker.py:138-160: Supervisor.update_nn + clear_unique_states):
 * the launcher swaps in the new weights (blob: host float32, or device memory when device_blob,
 * e.g. after an RCCL broadcast) between two launches, so every pool batch runs on exactly one
 * network, then clears the duplicate filters if clear_unique_states.  Blocks until applied. */
int gz_runner_update_network(gz_runner* r, const float* blob, size_t count, int device_blob,
                             int clear_unique_states, double timeout_s);
/* After a roll: pool_batches[i] = batches of pool i launched on the previous network;
 * *launches_before = launches issued before the swap. */
int gz_runner_roll_info(gz_runner* r, long* pool_batches, int npools, long* launches_before);
/* wall milliseconds the launcher spent applying the last roll (the weight fold / pack and swap) */
double gz_runner_roll_apply_ms(gz_runner* r);
/* Per-game costs by the game's ordinal within its slot, summed over the runner's pools (struct
 * gz_ordinal_stats, include/gzero_engine.h); a snapshot, safe while the runner runs. */
struct gz_ordinal_stats;
int gz_runner_ordinal_stats(gz_runner* r, struct gz_ordinal_stats* out);
const char* gz_runner_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* GZERO_NN_H */
