"""GPU parity of the fused HIP forward (libgz_nn.so via its C-ABI) against the oracle.

Stated tolerance (bf16 MFMA operands, fp32 accumulate, fp32 residual stream and heads), measured
against the float64 reference semantics oracle/nn_ref.forward: per variant, 3x the max / mean abs
error measured on MI355X for these seeded inputs (profiles/r02c_gpu_tests.log), TOL_BF16 below.
The fp32-accuracy mode (split hi/lo operands) has its own, ~100x tighter tolerance (TOL_FP32).
and against the bf16-emulating oracle (same rounding points as the kernel, differing only in
accumulation order, which flips an occasional bf16 rounding of an activation; the flips compound
with depth):
    nets with <= 1 residual block: max |err| <= 2e-3, mean |err| <= 2e-5   (TOL_EMU_SHALLOW)
    deeper nets:                   max |err| <= 2e-2, mean |err| <= 5e-3   (TOL_EMU_DEEP)
Row results must be bit-identical regardless of batch size / slot (batch invariance, needed for
bit-exact PUCT visit counts under batching).
"""
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS, NetDesc
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
from oracle import nn_ref

# 3 x measured (max, mean) abs error vs the float64 oracle, bf16 mode (profiles/r02c_gpu_tests.log)
TOL_BF16 = {"cfg1": (6.4e-3, 1.4e-4), "cfg2": (7.5e-2, 9.3e-3), "b0_8x8": (2.6e-3, 1.6e-3),
            "leaky_v3_8x8": (1e-2, 9e-4), "nchw_6x6": (3.3e-3, 1e-3), "cfg3": (3.2e-3, 1e-3),
            "cfg4": (7e-4, 2.5e-5), "cfg5": (3.1e-3, 1.4e-3), "b2_13x13_f256": (1.3e-2, 2.4e-3),
            "b0_10x10_f256_v3": (1e-3, 4.1e-4), "legacy_v1_8x8": (8.7e-3, 1.1e-4), "x6_102_json": (5e-4, 2.5e-4)}
TOL_REF = TOL_BF16["cfg2"]
TOL_EMU_SHALLOW = (2e-3, 2e-5)
TOL_EMU_DEEP = (2e-2, 5e-3)

pytestmark = pytest.mark.gpu

VARIANTS = {
    "cfg1": BASELINE_CONFIGS[1]["desc"],
    "cfg2": BASELINE_CONFIGS[2]["desc"],
    "b0_8x8": NetDesc(5, 8, 8, 128, 0, [155, 155]),
    "leaky_v3_8x8": NetDesc(5, 8, 8, 64, 1, [65, 65], num_values=3, leaky_relu=True),
    "nchw_6x6": NetDesc(5, 6, 6, 128, 1, [81, 81], flatten_nchw=True),
    # BASELINE configs 3-5 (reversi 8x8 with the draw head; F = 256 nets on 13x13 / 10x10 boards,
    # the single-LDS-image kernels, 13x13 with the residual stream in a device scratch)
    "cfg3": BASELINE_CONFIGS[3]["desc"],
    "cfg4": BASELINE_CONFIGS[4]["desc"],
    "cfg5": BASELINE_CONFIGS[5]["desc"],
    "b2_13x13_f256": NetDesc(5, 13, 13, 256, 2, [170, 171], flatten_nchw=True),
    "b0_10x10_f256_v3": NetDesc(12, 10, 10, 256, 0, [3041, 3041], num_values=3, leaky_relu=True),
    # legacy v1 model files (x6_102.json): conv biases folded into BN, value BN, sigmoid value
    "legacy_v1_8x8": NetDesc(5, 8, 8, 128, 2, [155, 155], flatten_nchw=True, conv_bias=True, value_bn=True,
                             value_sigmoid=True),
}
# the reference's own model file breakthrough/models/x6_102.json as the importer reads it
# (tests/golden/keras_descs.json, nn/keras_model.py): 10 x 128 with the legacy flags
with open(os.path.join(os.path.dirname(__file__), "golden", "keras_descs.json")) as _f:
    VARIANTS["x6_102_json"] = NetDesc(**json.load(_f)["breakthrough/models/x6_102.json"]["desc"])
DEEP = {"cfg3", "cfg4", "cfg5", "x6_102_json"}       # residual gamma damped so the softmaxes do not saturate
BIG = {"cfg4", "cfg5", "b2_13x13_f256", "b0_10x10_f256_v3"}   # oracle batch sizes kept small


def _net(desc, seed, device, name=None):
    from galvanise_zero_amd._native import HipNet
    w = random_weights(desc, seed, bias_std=0.2, res_gamma=0.15 if name in DEEP else 1.0)
    net = HipNet(desc, device)
    net.set_weights(to_blob(w))
    return net, w


def _err(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return float(d.max()), float(d.mean())


@pytest.mark.parametrize("name", list(VARIANTS))
def test_forward_parity(name, hip_device):
    desc = VARIANTS[name]
    net, w = _net(desc, 7919, hip_device, name)
    tol_emu = TOL_EMU_SHALLOW if desc.residual_layers <= 1 else TOL_EMU_DEEP
    for n in ((1, 7, 19) if name in BIG else (1, 7, 64)):
        x = random_planes(desc, n, 100 + n)
        got = net.forward(x)
        ref = nn_ref.forward(desc, w, x)
        emu = nn_ref.forward_bf16_emulated(desc, w, x)
        for i, (g, r, e) in enumerate(zip(got, ref, emu)):
            assert g.shape == r.shape
            assert np.all(np.isfinite(g))
            er, ee = _err(g, r), _err(g, e)
            print("%s n=%d out%d  vs_ref max %.3g mean %.3g | vs_emu max %.3g mean %.3g"
                  % (name, n, i, er[0], er[1], ee[0], ee[1]))
            tol = TOL_BF16[name]
            assert er[0] <= tol[0] and er[1] <= tol[1], (name, n, i, er)
            assert ee[0] <= tol_emu[0] and ee[1] <= tol_emu[1], (name, n, i, ee)
            if not (desc.value_sigmoid and i == len(got) - 1):   # sigmoid values are independent
                np.testing.assert_allclose(g.sum(axis=1), 1.0, atol=1e-4)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4", "cfg5"])
def test_batch_invariance(name, hip_device):
    desc = VARIANTS[name]
    net, _ = _net(desc, 3, hip_device, name)
    x = random_planes(desc, 256, 9)
    full = net.forward(x)
    # same rows in a different batch composition / slot
    perm = np.random.default_rng(0).permutation(256)[:37]
    part = net.forward(x[perm])
    for a, b in zip(full, part):
        assert np.array_equal(a[perm], b)
    single = net.forward(x[5:6])
    for a, b in zip(full, single):
        assert np.array_equal(a[5:6], b)


def test_large_batch_and_timing(hip_device):
    desc = VARIANTS["cfg2"]
    net, w = _net(desc, 1, hip_device)
    x = random_planes(desc, 1024, 5)
    got = net.forward(x)
    ref = nn_ref.forward(desc, w, x[:16])
    for g, r in zip(got, ref):
        assert _err(g[:16], r)[0] <= TOL_REF[0]
    ms = net.last_kernel_ms()
    tflops = desc.flops_per_eval() * 1024 / (ms * 1e-3) / 1e12
    print("cfg2 N=1024 kernel %.3f ms  %.1f TFLOP/s" % (ms, tflops))
    assert ms > 0


@pytest.mark.parametrize("variant", ["11", "12", "21"])
def test_kernel_variants_identical(variant, hip_device, monkeypatch):
    """Every compiled trunk variant (boards per workgroup x workgroups per CU) computes each row
    with the same operations in the same order: outputs are bit-identical to the default's."""
    desc = VARIANTS["cfg2"]
    x = random_planes(desc, 33, 4)
    net, _ = _net(desc, 5, hip_device)
    base = net.forward(x)
    monkeypatch.setenv("GZ_KERNEL_VARIANT", variant)
    vnet, _ = _net(desc, 5, hip_device)
    for a, b in zip(base, vnet.forward(x)):
        assert np.array_equal(a, b)


# ---- fp32-accuracy mode (split hi/lo bf16 operands, three MFMAs per product) ------------------
# Stated tolerance against the float64 oracle (reference semantics), per output element and per
# row (KL divergence of each policy / value row from the oracle's):
# 3 x the worst measured over SPLIT (max 6.7e-5, mean 1.6e-5, KL 1.4e-7; profiles/r02c_gpu_tests.log)
TOL_FP32 = (2e-4, 5e-5)          # max |err|, mean |err|
TOL_FP32_KL = 5e-7               # max over rows of KL(oracle || kernel)
SPLIT = ["cfg1", "cfg2", "cfg3", "b0_8x8", "leaky_v3_8x8", "nchw_6x6", "legacy_v1_8x8", "x6_102_json",
         # F = 256 on 10 x 10 (single-image split kernel): amazons cfg5 and a leaky / draw-head net
         "cfg5", "b0_10x10_f256_v3",
         # F = 256 on 13 x 13 (two-pass split kernel, P = 2): hexLG13 cfg4 and a 2-block net
         "cfg4", "b2_13x13_f256"]


def _net_p(desc, seed, device, name, precision):
    from galvanise_zero_amd._native import HipNet
    w = random_weights(desc, seed, bias_std=0.2, res_gamma=0.15 if name in DEEP else 1.0)
    net = HipNet(desc, device, precision)
    net.set_weights(to_blob(w))
    return net, w


def _kl(ref, got):
    r = np.clip(ref.astype(np.float64), 1e-30, None)
    g = np.clip(got.astype(np.float64), 1e-30, None)
    return float((r * np.log(r / g)).sum(axis=1).max())


@pytest.mark.parametrize("name", SPLIT)
def test_forward_parity_fp32(name, hip_device):
    desc = VARIANTS[name]
    net, w = _net_p(desc, 7919, hip_device, name, "bf16x3")
    for n in ((1, 7, 19) if name in BIG else (1, 7, 64)):
        x = random_planes(desc, n, 100 + n)
        got = net.forward(x)
        ref = nn_ref.forward(desc, w, x)
        for i, (g, r) in enumerate(zip(got, ref)):
            er = _err(g, r)
            sig = desc.value_sigmoid and i == len(got) - 1
            kl = 0.0 if sig else _kl(r, g)
            print("fp32 %s n=%d out%d  vs_ref max %.3g mean %.3g kl %.3g" % (name, n, i, er[0], er[1], kl))
            assert er[0] <= TOL_FP32[0] and er[1] <= TOL_FP32[1], (name, n, i, er)
            assert kl <= TOL_FP32_KL, (name, n, i, kl)


def test_fp32_tolerance_detects_one_bf16_ulp(hip_device):
    """The fp32-mode tolerance is tight enough to see a one-bf16-ulp (2^-8 relative) change of
    one residual block's conv weights."""
    from galvanise_zero_amd._native import HipNet
    desc = VARIANTS["cfg2"]
    w = random_weights(desc, 7919, bias_std=0.2)
    wp = [(k, v * np.float32(1 + 2.0 ** -8) if k == "res2_conv1" else v) for k, v in w]
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(to_blob(wp))
    x = random_planes(desc, 64, 164)
    errs = [_err(g, r)[0] for g, r in zip(net.forward(x), nn_ref.forward(desc, w, x))]
    print("one-ulp perturbation: max errors", errs)
    assert max(errs) > TOL_FP32[0]


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_batch_invariance_fp32(name, hip_device):
    desc = VARIANTS[name]
    net, _ = _net_p(desc, 3, hip_device, name, "bf16x3")
    x = random_planes(desc, 300, 9)
    full = net.forward(x)
    perm = np.random.default_rng(0).permutation(300)[:37]
    for a, b in zip(full, net.forward(x[perm])):
        assert np.array_equal(a[perm], b)


# ---- generic geometry: the reference's own network templates on every BASELINE game -----------
# templates.nn_model_config_template (reference templates.py:21-71): small F=64 x 5 blocks,
# medium F=96 x 5, large F=96 x 10 (F=96 runs on the 128-filter kernels with zero channels); the
# board is a kernel argument (kernels compiled per 16-position tile count).
TOL_BF16_GEOM = (9e-2, 1.8e-2)   # bf16 mode: 3 x the worst measured over these 15 nets (max 0.030, mean 0.0061; profiles/r02g_gpu_tests.log)
GEOM_GAMES = ["breakthroughSmall", "breakthrough", "reversi", "hexLG13", "amazons_10x10"]


def _template_desc(game, hint):
    from galvanise_zero_amd.defs import templates
    from galvanise_zero_amd.nn.bases import GdlBasesTransformer
    from galvanise_zero_amd.nn.network import desc_from_conf
    from galvanise_zero_amd.sm import get_sm
    gen = templates.default_generation_desc(game, num_previous_states=1)
    t = GdlBasesTransformer(get_sm(game), gen)
    return desc_from_conf(templates.nn_model_config_template(game, hint, t), gen)


@pytest.mark.parametrize("hint", ["small", "medium", "large"])
@pytest.mark.parametrize("game", GEOM_GAMES)
def test_template_geometries(game, hint, hip_device):
    from galvanise_zero_amd._native import HipNet
    desc = _template_desc(game, hint)
    w = random_weights(desc, 7919, bias_std=0.2, res_gamma=0.15 if desc.residual_layers > 6 else 1.0)
    x = random_planes(desc, 9, 31)
    ref = nn_ref.forward(desc, w, x)
    modes = [("bf16", TOL_BF16_GEOM), ("bf16x3", TOL_FP32)]   # (split beyond 8 x 8: the two-pass kernel)
    for precision, tol in modes:
        net = HipNet(desc, hip_device, precision)
        net.set_weights(to_blob(w))
        for i, (g, r) in enumerate(zip(net.forward(x), ref)):
            er = _err(g, r)
            print("geom %s/%s %s F=%d B=%d out%d vs_ref max %.3g mean %.3g" % (game, hint, precision, desc.cnn_filter_size,
                                                                             desc.residual_layers, i, er[0], er[1]))
            assert np.all(np.isfinite(g)) and g.shape == r.shape
            assert er[0] <= tol[0] and er[1] <= tol[1], (game, hint, precision, i, er)


@pytest.mark.parametrize("variant", ["11", "21", "22", "23", "24"])
def test_kernel_variants_identical_fp32(variant, hip_device, monkeypatch):
    """The split-precision kernels (one or two boards per workgroup; 22: two boards as two groups of
    four waves, trunk_kernel8) compute every row identically (33 rows: a dead board in the last
    workgroup)."""
    from galvanise_zero_amd._native import HipNet
    desc = VARIANTS["cfg2"]
    x = random_planes(desc, 33, 4)
    w = to_blob(random_weights(desc, 5, bias_std=0.2))
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(w)
    base = net.forward(x)
    monkeypatch.setenv("GZ_KERNEL_VARIANT", variant)
    vnet = HipNet(desc, hip_device, "bf16x3")
    vnet.set_weights(w)
    for a, b in zip(base, vnet.forward(x)):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("n", [512, 1031])
@pytest.mark.parametrize("variant", ["22", "23", "24"])
def test_wave_group_kernel_identical_at_bench_size(variant, n, hip_device, monkeypatch):
    """The wave-group kernels (variant 22, trunk_kernel8: one board per group of four waves; 23,
    trunk_kernel_h2: one board per group of two waves, each half the board's channels; 24,
    trunk_kernel_w8: one group of eight waves, each half of a 4-wave layout's channels) against the
    two-board kernel (21) at launch sizes of the bench (one and three workgroup rounds): bit-identical."""
    from galvanise_zero_amd._native import HipNet
    desc = VARIANTS["cfg2"]
    x = random_planes(desc, n, 6)
    w = to_blob(random_weights(desc, 7921))
    outs = []
    for v in ("21", variant):
        monkeypatch.setenv("GZ_KERNEL_VARIANT", v)
        net = HipNet(desc, hip_device, "bf16x3")
        net.set_weights(w)
        outs.append(net.forward(x))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_split_precision_against_fp32(hip_device):
    """What the bench's dtype ("bf16x3 split") means numerically: on the bench's net and weights
    (cfg2, random_weights(desc, 7921)) at a 1,024-row launch, the split kernel's error against the
    float64 oracle (model.py:154-296) next to a true IEEE fp32 forward's (torch-CPU float32,
    oracle/nn_torch.py) and the bf16 kernel's.  Measured on MI355X: profiles/r03s_gpu_tests.log.
    The split kernel sits between the two: ~16 significant bits per operand (hi + lo bf16, lo*lo
    dropped) against fp32's 24 and bf16's 8."""
    from galvanise_zero_amd._native import HipNet
    from oracle.nn_torch import TorchCPUNet
    desc = VARIANTS["cfg2"]
    w = random_weights(desc, 7921)
    x = random_planes(desc, 1024, 11)
    ref = nn_ref.forward(desc, w, x)
    t32 = TorchCPUNet(desc, w).predict_on_batch(x)
    errs = {"fp32 (torch-CPU)": [np.abs(np.asarray(g, np.float64) - r).max() for g, r in zip(t32, ref)]}
    for precision in ("bf16x3", "bf16"):
        net = HipNet(desc, hip_device, precision)
        net.set_weights(to_blob(w))
        errs["split" if precision == "bf16x3" else "bf16"] = [np.abs(g - r).max() for g, r in zip(net.forward(x), ref)]
    for k, v in errs.items():
        print("precision %-18s max |err| vs float64 oracle per output: %s" % (k, " ".join("%.3g" % e for e in v)))
    split, f32, b16 = max(errs["split"]), max(errs["fp32 (torch-CPU)"]), max(errs["bf16"])
    # measured on MI355X (profiles/r03s_gpu_tests.log): fp32 5.7e-6, split 2.0e-4, bf16 5.9e-2 (the
    # undamped bench weights at 1,024 rows); the split's bound is the stated cfg2 tolerance
    # (galvanise_zero_amd/nn/tolerance.py: 3x the max over 10 seeds, profiles/r04a_split_error_dist.json)
    from galvanise_zero_amd.nn.tolerance import SPLIT_TOLERANCE
    assert f32 < split < b16
    assert split <= SPLIT_TOLERANCE["cfg2"]["max"] and split * 20 < b16


# ---- initial-conv widths: the im2col row of a 3x3 initial conv holds K0 = 9 C (rounded up to 32)
# bf16 values; its chunk swizzle must stay inside the row for every K0 (rounds 1-4 sent chunks of
# K0 = 96 / 160 / 224 rows into the next position's, which the loose bf16 tolerances hid)
# 3 x the worst measured (profiles/r05c_large_board_errors.log): bf16 2.4e-3 / 9.1e-4, split 5.6e-6 / 2.6e-6
TOL_K0 = {"bf16": (7.3e-3, 2.8e-3), "bf16x3": (1.7e-5, 7.9e-6)}


@pytest.mark.parametrize("precision", ["bf16", "bf16x3"])
@pytest.mark.parametrize("hw", [8, 13])
@pytest.mark.parametrize("C", [3, 5, 9, 12, 15, 24])
def test_initial_conv_widths(C, hw, precision, hip_device):
    from galvanise_zero_amd._native import HipNet
    desc = NetDesc(C, hw, hw, 64, 1, [hw * hw + 1, hw * hw + 1])
    w = random_weights(desc, 7919, bias_std=0.2)
    try:
        net = HipNet(desc, hip_device, precision)
    except RuntimeError as e:   # 24 planes on 13 x 13 in split precision: the im2col staging exceeds the LDS
        assert (C, hw, precision) == (24, 13, "bf16x3") and "LDS" in str(e), e
        return
    net.set_weights(to_blob(w))
    x = random_planes(desc, 7, 100)
    for i, (g, r) in enumerate(zip(net.forward(x), nn_ref.forward(desc, w, x))):
        er = _err(g, r)
        print("k0 C=%d %dx%d %s out%d max %.3g mean %.3g" % (C, hw, hw, precision, i, er[0], er[1]))
        assert er[0] <= TOL_K0[precision][0] and er[1] <= TOL_K0[precision][1], (C, hw, precision, i, er)
