"""ctypes bindings of the in-tree native libraries (include/gzero_nn.h, include/gzero_engine.h).

The product path has no fallback: if a library is missing or fails to load, the call raises.
Libraries live in galvanise_zero_amd/lib/ (built by galvanise_zero_amd/csrc/Makefile).
"""

import ctypes
import os

import numpy as np

LIB_DIR = os.environ.get("GZ_LIB_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")   # GZ_LIB_DIR: A/B builds (tools/)
GZ_MAX_ROLES = 4

_libs = {}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name):
    return os.path.join(LIB_DIR, name)


def _load(name):
    lib = _libs.get(name)
    if lib is None:
        path = lib_path(name)
        if not os.path.exists(path):
            raise NativeLibraryMissing("native library %s not built (run __graft_entry__.build() or "
                                       "make -C galvanise_zero_amd/csrc)" % path)
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _libs[name] = lib
    return lib


###############################################################################
# libgz_nn.so

class GzNetDesc(ctypes.Structure):
    _fields_ = [("input_channels", ctypes.c_int),
                ("input_columns", ctypes.c_int),
                ("input_rows", ctypes.c_int),
                ("cnn_filter_size", ctypes.c_int),
                ("cnn_kernel_size", ctypes.c_int),
                ("residual_layers", ctypes.c_int),
                ("role_count", ctypes.c_int),
                ("policy_dist_count", ctypes.c_int * GZ_MAX_ROLES),
                ("value_hidden_size", ctypes.c_int),
                ("num_values", ctypes.c_int),
                ("leaky_relu", ctypes.c_int),
                ("flatten_nchw", ctypes.c_int),
                ("conv_bias", ctypes.c_int),
                ("value_bn", ctypes.c_int),
                ("value_sigmoid", ctypes.c_int),
                ("precision", ctypes.c_int),
                ("resnet_v2", ctypes.c_int),
                ("initial_kernel", ctypes.c_int),
                ("initial_bn", ctypes.c_int),
                ("se_units", ctypes.c_int),
                ("global_pooling_value", ctypes.c_int),
                ("concat_all_layers", ctypes.c_int)]

GZ_PRECISION_BF16 = 1
GZ_PRECISION_SPLIT = 3
# "bf16x3" (alias "split"): each fp32 operand as bf16 hi + lo, three MFMAs per product, ~16
# significant bits per operand -- fp32-CLASS, not IEEE fp32: on the headline cfg2 batch its error
# against the float64 oracle is ~35x an IEEE fp32 forward's (nn/tolerance.py).  "fp32" is the
# pre-round-6 name of the same mode, kept as a deprecated alias.
PRECISIONS = {"bf16": GZ_PRECISION_BF16, "bf16x3": GZ_PRECISION_SPLIT, "split": GZ_PRECISION_SPLIT,
              "fp32": GZ_PRECISION_SPLIT}


def canonical_precision(precision):
    """The arithmetic mode's canonical name ("bf16" or "bf16x3"); "split" and the deprecated "fp32"
    name bf16x3."""
    if precision not in PRECISIONS:
        raise ValueError("precision %r: one of bf16, bf16x3 (alias split; fp32 is deprecated)" % (precision,))
    if precision == "fp32":
        import warnings
        warnings.warn('precision "fp32" selects the bf16x3 split mode (three bf16 MFMAs per product, '
                      'fp32-class, not IEEE fp32): use "bf16x3"', DeprecationWarning, stacklevel=3)
    return "bf16" if PRECISIONS[precision] == GZ_PRECISION_BF16 else "bf16x3"


_FP = ctypes.POINTER(ctypes.c_float)
GZ_MAX_SEGMENTS = 32


class GzSegment(ctypes.Structure):
    """gz_segment (include/gzero_nn.h): one run of boards of a segmented launch."""
    _fields_ = [("rows", ctypes.c_int),
                ("planes", ctypes.c_void_p),
                ("policies", ctypes.c_void_p * GZ_MAX_ROLES),
                ("values", ctypes.c_void_p)]


def nn_lib():
    lib = _load("libgz_nn.so")
    if not getattr(lib, "_gz_typed", False):
        lib.gz_net_create.restype = ctypes.c_void_p
        lib.gz_net_create.argtypes = [ctypes.POINTER(GzNetDesc), ctypes.c_int]
        lib.gz_net_destroy.argtypes = [ctypes.c_void_p]
        lib.gz_net_weight_count.restype = ctypes.c_size_t
        lib.gz_net_weight_count.argtypes = [ctypes.c_void_p]
        lib.gz_net_set_weights.argtypes = [ctypes.c_void_p, _FP, ctypes.c_size_t]
        lib.gz_net_set_weights_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.gz_net_last_roll_ms.restype = ctypes.c_double
        lib.gz_net_last_roll_ms.argtypes = [ctypes.c_void_p]
        lib.gz_net_copy_weight_image.restype = ctypes.c_size_t
        lib.gz_net_copy_weight_image.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.gz_net_forward.argtypes = [ctypes.c_void_p, _FP, ctypes.c_int,
                                       ctypes.POINTER(_FP), _FP]
        lib.gz_net_forward_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.c_void_p]
        lib.gz_net_forward_segments.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(GzSegment),
                                                ctypes.c_int]
        lib.gz_net_last_kernel_ms.restype = ctypes.c_float
        lib.gz_net_last_kernel_ms.argtypes = [ctypes.c_void_p]
        lib.gz_net_stamp_avg.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.gz_net_flops_per_eval.restype = ctypes.c_double
        lib.gz_net_flops_per_eval.argtypes = [ctypes.c_void_p]
        lib.gz_net_heads_fused.restype = ctypes.c_int
        lib.gz_net_heads_fused.argtypes = [ctypes.c_void_p]
        lib.gz_net_set_output_logits.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.gz_net_kernel_name.restype = ctypes.c_char_p
        lib.gz_net_kernel_name.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.gz_net_large_min_rows.restype = ctypes.c_int
        lib.gz_net_large_min_rows.argtypes = [ctypes.c_void_p]
        lib.gz_nn_last_error.restype = ctypes.c_char_p
        lib._gz_typed = True
    return lib


def make_net_desc(desc, precision=GZ_PRECISION_BF16):
    d = GzNetDesc()
    d.precision = precision
    d.input_channels = desc.input_channels
    d.input_columns = desc.input_columns
    d.input_rows = desc.input_rows
    d.cnn_filter_size = desc.cnn_filter_size
    d.cnn_kernel_size = desc.cnn_kernel_size
    d.residual_layers = desc.residual_layers
    d.role_count = len(desc.policy_dist_count)
    for i, p in enumerate(desc.policy_dist_count):
        d.policy_dist_count[i] = p
    d.value_hidden_size = desc.value_hidden_size
    d.num_values = desc.num_values
    d.leaky_relu = int(desc.leaky_relu)
    d.conv_bias = int(getattr(desc, "conv_bias", False))
    d.value_bn = int(getattr(desc, "value_bn", False))
    d.value_sigmoid = int(getattr(desc, "value_sigmoid", False))
    d.flatten_nchw = int(desc.flatten_nchw)
    d.resnet_v2 = int(getattr(desc, "resnet_v2", False))
    d.initial_kernel = int(desc.initial_kernel) if hasattr(desc, "initial_kernel") else 0
    d.initial_bn = int(getattr(desc, "initial_bn", True))
    d.se_units = int(getattr(desc, "se_units", 0))
    d.global_pooling_value = int(getattr(desc, "global_pooling_value", False))
    d.concat_all_layers = int(getattr(desc, "concat_all_layers", False))
    return d


def _fptr(a):
    return a.ctypes.data_as(_FP)


class HipNet(object):
    """Owner of a gz_net handle: the MI355X forward of one network on one device.
    precision: "bf16" (bf16 operands) or "bf16x3" (alias "split"; hi/lo bf16 operands, three MFMAs
    per product: fp32-class accuracy -- about 35x an IEEE fp32 forward's error on cfg2 -- not IEEE
    fp32, include/gzero_nn.h GZ_PRECISION_SPLIT).  "fp32" is a deprecated alias of "bf16x3";
    self.precision holds the canonical name."""

    def __init__(self, desc, device=0, precision="bf16"):
        self.lib = nn_lib()
        self.desc = desc
        self.precision = canonical_precision(precision)
        self._cdesc = make_net_desc(desc, PRECISIONS[self.precision])
        self.handle = self.lib.gz_net_create(ctypes.byref(self._cdesc), device)
        if not self.handle:
            raise RuntimeError("gz_net_create failed: %s" % self.lib.gz_nn_last_error().decode())
        self.weight_count = self.lib.gz_net_weight_count(self.handle)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed: %s" % (what, self.lib.gz_nn_last_error().decode()))

    def set_weights(self, blob):
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        if blob.size != self.weight_count:
            raise ValueError("weight blob has %d floats, network expects %d" % (blob.size, self.weight_count))
        self._check(self.lib.gz_net_set_weights(self.handle, _fptr(blob), blob.size), "gz_net_set_weights")

    def set_weights_device(self, ptr, count):
        self._check(self.lib.gz_net_set_weights_device(self.handle, ctypes.c_void_p(ptr), count),
                    "gz_net_set_weights_device")

    def last_roll_ms(self):
        """Device milliseconds of the last set_weights_device (BN fold + bf16 pack kernels)."""
        return self.lib.gz_net_last_roll_ms(self.handle)

    def weight_image(self):
        """The packed device weight image as bytes (diagnostics: host and device packing compare)."""
        n = self.lib.gz_net_copy_weight_image(self.handle, None, 0)
        buf = np.empty(n, dtype=np.uint8)
        got = self.lib.gz_net_copy_weight_image(self.handle, buf.ctypes.data, n)
        if got != n:
            raise RuntimeError("gz_net_copy_weight_image failed")
        return buf

    def forward(self, planes):
        d = self.desc
        planes = np.ascontiguousarray(planes, dtype=np.float32)
        n = planes.shape[0]
        assert planes.size == n * d.input_channels * d.input_columns * d.input_rows
        pols = [np.empty((n, p), dtype=np.float32) for p in d.policy_dist_count]
        val = np.empty((n, d.num_values), dtype=np.float32)
        arr = (_FP * len(pols))(*[_fptr(p) for p in pols])
        self._check(self.lib.gz_net_forward(self.handle, _fptr(planes), n, arr, _fptr(val)),
                    "gz_net_forward")
        return pols + [val]

    def forward_device(self, stream, d_planes, n, d_policies, d_values):
        arr = (ctypes.c_void_p * len(d_policies))(*d_policies)
        self._check(self.lib.gz_net_forward_device(self.handle, ctypes.c_void_p(stream),
                                                   ctypes.c_void_p(d_planes), n, arr,
                                                   ctypes.c_void_p(d_values)),
                    "gz_net_forward_device")

    def forward_segments(self, stream, segments):
        """Asynchronous segmented launch on `stream`: segments = [(rows, planes_ptr, [policy_ptr per
        role], values_ptr)]; pointers are device or pinned host addresses."""
        if not 1 <= len(segments) <= GZ_MAX_SEGMENTS:
            raise ValueError("1..%d segments" % GZ_MAX_SEGMENTS)
        segs = (GzSegment * len(segments))()
        for s, (rows, planes, pols, vals) in zip(segs, segments):
            s.rows = rows
            s.planes = planes
            for r, p in enumerate(pols):
                s.policies[r] = p
            s.values = vals
        self._check(self.lib.gz_net_forward_segments(self.handle, ctypes.c_void_p(stream), segs, len(segments)),
                    "gz_net_forward_segments")

    def last_kernel_ms(self):
        return self.lib.gz_net_last_kernel_ms(self.handle)

    def set_output_logits(self, on=True):
        """Diagnostics: later forwards return the heads' pre-activation outputs (logits)."""
        self._check(self.lib.gz_net_set_output_logits(self.handle, int(bool(on))), "gz_net_set_output_logits")

    def stamp_avg(self):
        out = (ctypes.c_double * 8)()
        self.lib.gz_net_stamp_avg(self.handle, out)
        return list(out)

    def flops_per_eval(self):
        return self.lib.gz_net_flops_per_eval(self.handle)

    def kernel_name(self, large):
        """The trunk kernel of small (below large_min_rows) / large launches, as rocprofv3 names it."""
        return self.lib.gz_net_kernel_name(self.handle, int(bool(large))).decode()

    def large_min_rows(self):
        return self.lib.gz_net_large_min_rows(self.handle)

    def heads_fused(self):
        """True when the large trunk variant runs the dense heads itself (no heads_kernel launch)."""
        return bool(self.lib.gz_net_heads_fused(self.handle))

    def close(self):
        if self.handle:
            self.lib.gz_net_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


###############################################################################
# libgz_engine.so

class GzPuctConfig(ctypes.Structure):
    _fields_ = [("verbose", ctypes.c_int),
                ("puct_constant", ctypes.c_float),
                ("puct_constant_root", ctypes.c_float),
                ("dirichlet_noise_pct", ctypes.c_float),
                ("noise_policy_squash_pct", ctypes.c_float),
                ("noise_policy_squash_prob", ctypes.c_float),
                ("choose", ctypes.c_int),
                ("max_dump_depth", ctypes.c_int),
                ("random_scale", ctypes.c_float),
                ("temperature", ctypes.c_float),
                ("depth_temperature_start", ctypes.c_int),
                ("depth_temperature_increment", ctypes.c_float),
                ("depth_temperature_stop", ctypes.c_int),
                ("depth_temperature_max", ctypes.c_float),
                ("fpu_prior_discount", ctypes.c_float),
                ("fpu_prior_discount_root", ctypes.c_float),
                ("top_visits_best_guess_converge_ratio", ctypes.c_float),
                ("think_time", ctypes.c_float),
                ("converged_visits", ctypes.c_int),
                ("batch_size", ctypes.c_int),
                ("use_legals_count_draw", ctypes.c_int),
                ("backup_finalised", ctypes.c_int),
                ("lookup_transpositions", ctypes.c_int),
                ("evaluation_multiplier_to_convergence", ctypes.c_float), ("spin_yield_playouts", ctypes.c_int)]


class GzSelfPlayConfig(ctypes.Structure):
    _fields_ = [("oscillate_sampling_pct", ctypes.c_float),
                ("temperature_for_policy", ctypes.c_float),
                ("puct_config", GzPuctConfig),
                ("evals_per_move", ctypes.c_int),
                ("resign0_score_probability", ctypes.c_float),
                ("resign0_pct", ctypes.c_float),
                ("resign1_score_probability", ctypes.c_float),
                ("resign1_pct", ctypes.c_float),
                ("abort_max_length", ctypes.c_int),
                ("number_repeat_states_draw", ctypes.c_int),
                ("repeat_states_score", ctypes.c_float),
                ("run_to_end_pct", ctypes.c_float),
                ("run_to_end_evals", ctypes.c_int),
                ("run_to_end_puct_config", GzPuctConfig),
                ("run_to_end_early_score", ctypes.c_float),
                ("run_to_end_minimum_game_depth", ctypes.c_int)]


class GzPoolStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_long) for n in (
        "games_started", "games_completed", "games_with_samples", "samples", "no_samples", "dupes",
        "resigns", "false_positive_resigns0", "false_positive_resigns1", "early_run_to_ends",
        "aborts_game_length", "evaluations", "polls", "completed_game_evals", "tree_playouts", "transpositions")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


GZ_ORDINALS, GZ_COST_HIST = 8, 32


class GzOrdinalStats(ctypes.Structure):
    """gz_ordinal_stats (include/gzero_engine.h): per-game cost by the game's ordinal in its slot."""
    _fields_ = [(n, ctypes.c_long * GZ_ORDINALS) for n in ("games", "evals", "tree_playouts", "moves", "spin_epochs")] + \
               [("engine_s", ctypes.c_double * GZ_ORDINALS), ("cost_hist", ctypes.c_long * GZ_COST_HIST),
                ("inflight_games", ctypes.c_long), ("inflight_engine_s", ctypes.c_double),
                ("inflight_evals", ctypes.c_long), ("inflight_games_ord", ctypes.c_long * GZ_ORDINALS),
                ("inflight_engine_s_ord", ctypes.c_double * GZ_ORDINALS),
                ("inflight_evals_ord", ctypes.c_long * GZ_ORDINALS)]

    def as_dict(self):
        out = {}
        for n, _ in self._fields_:
            v = getattr(self, n)
            out[n] = list(v) if hasattr(v, "__len__") else v
        return out


def set_verify_fastpath(on):
    """Run-time GZ_VERIFY_FASTPATH (process-wide); returns the previous setting."""
    return bool(engine_lib().gz_engine_set_verify_fastpath(1 if on else 0))


def verified_decisions():
    return int(engine_lib().gz_engine_verified_decisions())


_VP = ctypes.c_void_p
_U64P = ctypes.POINTER(ctypes.c_uint64)
_IP = ctypes.POINTER(ctypes.c_int)

_ENGINE_SIGS = {
    "gz_engine_last_error": (ctypes.c_char_p, []),
    "gz_free": (None, [_VP]),
    "gz_sm_create": (_VP, [ctypes.c_char_p]),
    "gz_sm_destroy": (None, [_VP]),
    "gz_sm_role_count": (ctypes.c_int, [_VP]),
    "gz_sm_num_bases": (ctypes.c_int, [_VP]),
    "gz_sm_num_words": (ctypes.c_int, [_VP]),
    "gz_sm_action_count": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_sm_base_name": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "gz_sm_role_name": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "gz_sm_legal_to_move": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "gz_sm_initial_state": (ctypes.c_int, [_VP, _U64P]),
    "gz_sm_update_bases": (ctypes.c_int, [_VP, _U64P]),
    "gz_sm_legal_count": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_sm_legal": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int]),
    "gz_sm_is_terminal": (ctypes.c_int, [_VP]),
    "gz_sm_goal_value": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_sm_next_state": (ctypes.c_int, [_VP, _IP, _U64P]),
    "gz_transformer_create": (_VP, [ctypes.c_int] * 5 + [_IP, ctypes.c_int]),
    "gz_transformer_destroy": (None, [_VP]),
    "gz_transformer_add_board_base": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int]),
    "gz_transformer_add_control_base": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_float]),
    "gz_transformer_total_size": (ctypes.c_int, [_VP]),
    "gz_transformer_to_channels": (ctypes.c_int, [_VP, _U64P, ctypes.POINTER(_U64P), ctypes.c_int, _FP]),
    "gz_supervisor_create": (_VP, [_VP, _VP, ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int]),
    "gz_supervisor_destroy": (None, [_VP]),
    "gz_supervisor_cancel": (ctypes.c_int, [_VP]),
    "gz_supervisor_start_self_play": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.POINTER(GzSelfPlayConfig)]),
    "gz_supervisor_poll": (_FP, [_VP, ctypes.c_int, ctypes.POINTER(_FP), ctypes.c_int, _IP]),
    "gz_supervisor_fetch_samples": (_VP, [_VP]),
    "gz_supervisor_add_unique_state": (ctypes.c_int, [_VP, _U64P]),
    "gz_supervisor_clear_unique_states": (ctypes.c_int, [_VP]),
    "gz_supervisor_stats": (ctypes.c_int, [_VP, ctypes.POINTER(GzPoolStats)]),
    "gz_supervisor_set_sample_interval": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_player_create": (_VP, [_VP, _VP, ctypes.POINTER(GzPuctConfig), ctypes.c_uint64]),
    "gz_player_destroy": (None, [_VP]),
    "gz_player_reset": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_player_apply_move": (ctypes.c_int, [_VP, _IP]),
    "gz_player_move": (ctypes.c_int, [_VP, _U64P, ctypes.c_int, ctypes.c_double]),
    "gz_player_get_move": (ctypes.c_int, [_VP, ctypes.c_int, _IP, _FP, _IP]),
    "gz_player_update_config": (ctypes.c_int, [_VP, ctypes.c_double, ctypes.c_int, ctypes.c_int]),
    "gz_player_balance_moves": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_player_tree_debug": (_VP, [_VP, ctypes.c_int]),
    "gz_player_poll": (_FP, [_VP, ctypes.c_int, ctypes.POINTER(_FP), ctypes.c_int, _IP]),
    "gz_player_root_children": (ctypes.c_int, [_VP, _IP, ctypes.POINTER(ctypes.c_uint32), _FP, ctypes.c_int]),
    "gz_unique_states_create": (_VP, [_VP, _VP, ctypes.c_int]),
    "gz_unique_states_destroy": (None, [_VP]),
    "gz_unique_states_clear": (ctypes.c_int, [_VP]),
    "gz_pool_clear_unique_states": (ctypes.c_int, [_VP]),
    "gz_pool_cancel": (ctypes.c_int, [_VP]),
    "gz_pool_create": (_VP, [_VP, _VP, ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_long, _VP,
                             _FP, ctypes.POINTER(_FP), _FP]),
    "gz_pool_destroy": (None, [_VP]),
    "gz_pool_start": (ctypes.c_int, [_VP, ctypes.POINTER(GzSelfPlayConfig)]),
    "gz_pool_poll": (ctypes.c_int, [_VP, ctypes.c_int]),
    "gz_pool_get_stats": (ctypes.c_int, [_VP, ctypes.POINTER(GzPoolStats)]),
    "gz_pool_fetch_samples": (_VP, [_VP]),
    "gz_pool_fetch_samples_n": (_VP, [_VP, ctypes.POINTER(ctypes.c_long)]),
    "gz_pool_take_sample_count": (ctypes.c_long, [_VP]),
    "gz_pool_add_ordinal_stats": (ctypes.c_int, [_VP, _VP]),
    "gz_engine_set_verify_fastpath": (ctypes.c_int, [ctypes.c_int]),
    "gz_engine_verified_decisions": (ctypes.c_long, []),
    "gz_engine_build_info": (ctypes.c_char_p, []),
}


def engine_lib():
    lib = _load("libgz_engine.so")
    if not getattr(lib, "_gz_typed", False):
        for name, (res, args) in _ENGINE_SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        lib._gz_typed = True
    return lib


def engine_error():
    return engine_lib().gz_engine_last_error().decode()


def take_string(ptr):
    """Copy and free a malloc'd C string returned by the engine (None for NULL)."""
    if not ptr:
        return None
    s = ctypes.string_at(ptr).decode()
    engine_lib().gz_free(ptr)
    return s


_CHOOSE = {"choose_top_visits": 0, "choose_temperature": 1}


def _get(conf, name, default):
    """Read a config field from an attrs record or a dict; missing keys keep the default (the
    reference's createSelfPlayConfig reads keys Python never sets, common.cpp:154-155)."""
    if isinstance(conf, dict):
        return conf.get(name, default)
    return getattr(conf, name, default)


def make_puct_config(conf):
    from .defs import confs
    d = confs.PUCTEvaluatorConfig()
    c = GzPuctConfig()
    for name, ctype in GzPuctConfig._fields_:
        v = _get(conf, name, getattr(d, name, 0))
        if name == "choose":
            if isinstance(v, str):
                v = _CHOOSE.get(v, 0)
        setattr(c, name, int(v) if ctype is ctypes.c_int else float(v))
    return c


def make_selfplay_config(conf):
    from .defs import confs
    d = confs.SelfPlayConfig()
    c = GzSelfPlayConfig()
    for name, ctype in GzSelfPlayConfig._fields_:
        if name in ("puct_config", "run_to_end_puct_config"):
            setattr(c, name, make_puct_config(_get(conf, name, getattr(d, name))))
            continue
        default = {"number_repeat_states_draw": -1, "repeat_states_score": 0.5}.get(name)
        if default is None:
            default = getattr(d, name)
        v = _get(conf, name, default)
        setattr(c, name, int(v) if ctype is ctypes.c_int else float(v))
    return c


###############################################################################
# runner (libgz_nn.so, runner.hip)

class GzRunnerConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("num_threads", ctypes.c_int), ("pools_per_thread", ctypes.c_int),
                ("batch_size", ctypes.c_int), ("seed", ctypes.c_ulonglong), ("game_index_base", ctypes.c_long),
                ("per_pool_unique_states", ctypes.c_int), ("keep_samples", ctypes.c_int),
                ("max_launch_rows", ctypes.c_int), ("min_launch_rows", ctypes.c_int),
                ("max_launch_wait_us", ctypes.c_int)]


class GzRunnerStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_long), ("rows", ctypes.c_long), ("kernel_ms", ctypes.c_double),
                ("trunk_ms", ctypes.c_double),
                ("kernel_launches", ctypes.c_long), ("games_completed", ctypes.c_long),
                ("games_with_samples", ctypes.c_long), ("samples", ctypes.c_long), ("no_samples", ctypes.c_long),
                ("resigns", ctypes.c_long), ("aborts", ctypes.c_long), ("dupes", ctypes.c_long),
                ("segments", ctypes.c_long), ("completed_game_evals", ctypes.c_long),
                ("large_launches", ctypes.c_long), ("large_rows", ctypes.c_long), ("large_trunk_ms", ctypes.c_double),
                ("engine_idle_ms", ctypes.c_double), ("tree_playouts", ctypes.c_long),
                ("large_rounds", ctypes.c_long), ("split_launches", ctypes.c_long)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def runner_lib():
    lib = nn_lib()
    if not getattr(lib, "_gz_runner_typed", False):
        lib.gz_runner_create.restype = _VP
        lib.gz_runner_create.argtypes = [_VP, _VP, _VP, ctypes.POINTER(GzRunnerConfig),
                                         ctypes.POINTER(GzSelfPlayConfig), _IP, ctypes.c_int, ctypes.c_int]
        lib.gz_runner_start.argtypes = [_VP]
        lib.gz_runner_wait_batches.argtypes = [_VP, ctypes.c_long, ctypes.c_double]
        lib.gz_runner_wait_rows.argtypes = [_VP, ctypes.c_long, ctypes.c_double]
        lib.gz_runner_fetch_samples.restype = _VP
        lib.gz_runner_fetch_samples.argtypes = [_VP]
        lib.gz_runner_stats_get.argtypes = [_VP, ctypes.POINTER(GzRunnerStats)]
        lib.gz_runner_stop.argtypes = [_VP]
        lib.gz_runner_destroy.argtypes = [_VP]
        lib.gz_runner_last_error.restype = ctypes.c_char_p
        lib.gz_runner_clear_unique_states.argtypes = [_VP]
        lib.gz_runner_update_network.argtypes = [_VP, _VP, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        lib.gz_runner_roll_apply_ms.restype = ctypes.c_double
        lib.gz_runner_roll_apply_ms.argtypes = [_VP]
        lib.gz_runner_roll_info.argtypes = [_VP, ctypes.POINTER(ctypes.c_long), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_long)]
        lib.gz_runner_ordinal_stats.argtypes = [_VP, ctypes.POINTER(GzOrdinalStats)]
        lib._gz_runner_typed = True
    return lib


def engine_build_info():
    """How libgz_engine.so was built: "pgo=<use|none|stale|gen> march=<...>" (csrc/Makefile)."""
    return engine_lib().gz_engine_build_info().decode()
