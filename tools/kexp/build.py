"""Diagnostic builds of the F = 128, 8x8 split trunk kernel (not product code): copies csrc/nn to
/tmp, applies one source patch per experiment, and builds libgz_nn.so (only the F = 128 / PT = 4
instantiations; the other filter counts are stubbed) into tools/kexp/lib_<name>/ next to a copy of
libgz_engine.so.  Timing on the GPU box: GZ_LIB_DIR=tools/kexp/lib_<name> python tools/kernel_variants.py ...

  base         unpatched (same-box reference)
  nostore      the residual epilogues compute but do not write the next LDS image (epilogue ds_writes)
  l1weights    every weight-ring stage reads stage 0's fragments (weights from L1 instead of L2)
  unroll       the fully unrolled conv of round 2 instead of the looped one
  nobarrier    no workgroup barrier after the residual epilogues (results wrong; barrier cost)
  noaddr       every tap reads the centre tap's B addresses (no per-tap address arithmetic)
  noreads      no B-fragment LDS reads after each conv's first k-step
  siunroll     the single-image kernels' fully unrolled conv (round 3) instead of the looped one
  headsunroll  the dense heads' weight loops unrolled 128 (policy) / 64 (value) instead of 32
  noheads      the fused trunk kernels skip the dense heads (results wrong; their cost)
  nophaseb     the two-phase dense heads skip phase B (softmax / value waves; results wrong)
  ring6/ring12 the two-board split kernel's weight ring 6 / 12 stages deep instead of one tap (4)
  lounroll16   the two-pass kernel's lo-image copies 16 uint4 per thread in flight instead of 4
  nolocopy     the two-pass kernel skips the lo-image copies (results wrong; their cost)
  epion        the two-image kernels' epilogues inside the conv's last k-step instead of after it
  lodirectoff  the two-pass kernel's epilogues write the lo parts into the image and sweep them out
               (round-3 / r04n scheme) instead of straight to the scratch
  swapon       the split two-image epilogues store one 16-byte chunk half per lane after a lane swap
               instead of two 8-byte halves (kStoreSwap)
  a+b          both patches
  full_<name>  patch <name>, build every trunk instantiation (the deep configs' F = 256 kernels)
Usage: python tools/kexp/build.py base nostore ...
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "galvanise_zero_amd", "csrc", "nn")

STUB = r'''
#include "trunk_variants.h"
namespace gznn {
KernelChoice trunk_variant_f128(int pt, int v, int precision) {
    if (pt == 4) return variants<128, 4>(v, precision);
    return KernelChoice{};
}
KernelChoice trunk_variant_f64(int, int, int) { return KernelChoice{}; }
KernelChoice trunk_variant_f256(int, int, int) { return KernelChoice{}; }
KernelChoice trunk_variant_f64_v2(int, int, int) { return KernelChoice{}; }
KernelChoice trunk_variant_f128_v2(int, int, int) { return KernelChoice{}; }
}
'''


def patch(name, text):  # noqa: C901
    def rep(old, new, count=1):
        nonlocal text
        assert text.count(old) >= count, (name, old)
        text = text.replace(old, new)
    if name in ("base", "pad"):
        pass
    elif name == "nostore":
        rep("        *(uint2*)a = u;\n", "        if (npos < 0) *(uint2*)a = u;\n")
        rep("            *(uint2*)(a + G::HALF) = l;\n", "            if (npos < 0) *(uint2*)(a + G::HALF) = l;\n")
    elif name == "l1weights":
        rep("    const int s = gs < gmax ? gs : gmax;\n", "    const int s = (gs < gmax ? gs : gmax) & 0;\n")
    elif name == "nobarrier":
        # the two barriers closing the v1 residual epilogues (two-image kernels)
        rep("                store_act<F, PTN, P>(X1 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);\n"
            "            }\n        }\n        __syncthreads();\n",
            "                store_act<F, PTN, P>(X1 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);\n"
            "            }\n        }\n")
        rep("                store_act<F, PTN, P>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);\n"
            "            }\n        }\n        __syncthreads();\n    }\n",
            "                store_act<F, PTN, P>(X0 + (t / PT) * ACT, 16 * (t % PT) + li, co, v, NPOS);\n"
            "            }\n        }\n    }\n")
    elif name == "headsunroll":
        rep("#pragma unroll 32   // many weight loads in flight: the loop is L2-latency bound\n            for (int k = 0; k < K; ++k) {",
            "#pragma unroll 128\n            for (int k = 0; k < K; ++k) {")
        rep("#pragma unroll 32   // many weight loads in flight: the loop is L2-latency bound\n            for (int k = 0; k < VK; ++k) {",
            "#pragma unroll 64\n            for (int k = 0; k < VK; ++k) {")
    elif name in ("ring6", "ring12"):
        rep("                                  ? KC / KS\n", "                                  ? %s\n" % ("3 * KC / KS / 2" if name == "ring6" else "3 * KC / KS"))
        rep("                               (KC / KS) * KS * NFR * 4 <= 96)", "                               (KC / KS) * KS * NFR * 4 <= 96 && NB == 2)")
    elif name == "lounroll16":
        rep("#pragma unroll 4\n    for (int i = tid; i < n16; i += 256) {", "#pragma unroll 16\n    for (int i = tid; i < n16; i += 256) {")
    elif name == "nolocopy":
        rep("    for (int i = tid; i < n16; i += 256) {", "    for (int i = tid; i < n16 && npos < 0; i += 256) {")
    elif name == "epion":
        rep("constexpr bool kEpiInConv = false;", "constexpr bool kEpiInConv = true;")
    elif name == "lodirectoff":
        rep("constexpr bool kLoDirect = true;", "constexpr bool kLoDirect = false;")
    elif name == "swapon":
        rep("constexpr bool kStoreSwap = false;", "constexpr bool kStoreSwap = true;")
    elif name == "noheads":
        rep("        dense_heads<NBW, kThreads * NGR>(kp, fk, lg, wb0, nb);", "        if (nb < 0) dense_heads<NBW, kThreads * NGR>(kp, fk, lg, wb0, nb);")
    elif name == "nophaseb":
        rep("    const int ntask = R * nb + nb;\n", "    const int ntask = nb < 0 ? R * nb + nb : 0;\n")
    elif name == "siunroll":
        rep("    static constexpr bool LOOPSI = SI && NST % US == 0 && NST / US >= 2;\n",
            "    static constexpr bool LOOPSI = false;\n")
    elif name == "unroll":
        rep("    static constexpr bool LOOP = !SI && NST % U == 0 && NIT >= 2;\n", "    static constexpr bool LOOP = false;\n")
    elif name == "noaddr":
        rep("    const int dy = tap / 3 - 1, dx = tap % 3 - 1;\n", "    const int dy = 0, dx = 0;\n")
        rep("    const bool ok = (bd.tapmask[pt] >> tap) & 1;\n", "    const bool ok = (bd.tapmask[pt] >> 4) & 1;\n")
    elif name == "noreads":
        rep("        if (j + 1 < 9 * KC) {                  // B fragments of the next k-step (double buffer)\n",
            "        if (false) {\n")
        rep("                acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[j & 1][t][0], acc[ct][t], 0, 0, 0);\n",
            "                acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[0][t][0], acc[ct][t], 0, 0, 0);\n")
        rep("                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[j & 1][t][1], acc[ct][t], 0, 0, 0);\n",
            "                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[0][t][1], acc[ct][t], 0, 0, 0);\n")
        rep("                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[j & 1][t][0], acc[ct][t], 0, 0, 0);\n",
            "                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[0][t][0], acc[ct][t], 0, 0, 0);\n")
    elif name == "asmchain":
        # the looped conv's three split products of one (co tile, position tile) as ONE inline-asm
        # chain with dst == srcC (the accumulate-forwarding case: no interlock), instead of builtins
        # the register allocator renames (dst != srcC, copies at the loop top); s_nop 1 first (a VALU
        # write of an operand right before), s_nop 15 after each conv (VALU reads of the last D)
        rep("""                    acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[t][0], acc[ct][t], 0, 0, 0);
                    if constexpr (P2 == 2) {
                        const bf16x8 w_lo = ring.r[ST % R][k][ct * WP + 1];
                        acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[t][1], acc[ct][t], 0, 0, 0);
                        acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_lo, b[t][0], acc[ct][t], 0, 0, 0);
                    }
""", """                    if constexpr (P2 == 2) {
                        const bf16x8 w_lo = ring.r[ST % R][k][ct * WP + 1];
                        asm volatile("s_nop 1\\n\\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\\n\\t"
                                     "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\\n\\t"
                                     "v_mfma_f32_16x16x32_bf16 %0, %4, %2, %0"
                                     : "+a"(acc[ct][t]) : "v"(w_hi), "v"(b[t][0]), "v"(b[t][1]), "v"(w_lo));
                    } else {
                        acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_hi, b[t][0], acc[ct][t], 0, 0, 0);
                    }
""")
        rep("""                __builtin_amdgcn_sched_group_barrier(0x008, CT * (P2 == 2 ? 3 : 1), 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, P2, 0);                       // DS read
            }
        __builtin_amdgcn_sched_barrier(0);""", """            }
        __builtin_amdgcn_sched_barrier(0);""")
        rep("""        conv_iter<F, PTN, NB, P, WG>(X, ring, acc, b, wres, woff, gs0 + it * G::U, gmax, lane, bd, it * G::TPI,
                                 it == G::NIT - 1, std::make_integer_sequence<int, G::U>{});
""", """        conv_iter<F, PTN, NB, P, WG>(X, ring, acc, b, wres, woff, gs0 + it * G::U, gmax, lane, bd, it * G::TPI,
                                 it == G::NIT - 1, std::make_integer_sequence<int, G::U>{});
    asm volatile("s_nop 15" ::: "memory");
""")
    elif name == "asmchain_nonop":
        # asmchain without the leading s_nop 1 (the operands come from loads, not VALU writes)
        text = patch("asmchain", text)
        rep('asm volatile("s_nop 1\\n\\tv_mfma_f32_16x16x32_bf16', 'asm volatile("v_mfma_f32_16x16x32_bf16')
    elif "+" in name:
        for part in name.split("+"):
            text = patch(part, text)
    else:
        raise SystemExit("unknown experiment " + name)
    return text


def build(name):
    full = name.startswith("full_")
    work = "/tmp/kexp_" + name
    shutil.rmtree(work, ignore_errors=True)
    shutil.copytree(SRC, os.path.join(work, "nn"))
    os.makedirs(os.path.join(work, "include"), exist_ok=True)
    for h in ("gzero_nn.h", "gzero_engine.h"):
        shutil.copy(os.path.join(ROOT, "include", h), os.path.join(work, "include", h))
    nn = os.path.join(work, "nn")
    # the sources include ../../../include/...: mirror that depth
    for f in os.listdir(nn):
        p = os.path.join(nn, f)
        t = open(p).read().replace("../../../include/", "../include/")
        if f == "forward_kernel.h":
            t = patch(name[5:] if full else name, t)
        open(p, "w").write(t)
    if not full:
        open(os.path.join(nn, "trunk_exp.hip"), "w").write(STUB)
    out = os.path.join(ROOT, "tools", "kexp", "lib_" + name)
    os.makedirs(out, exist_ok=True)
    eng = os.path.join(out, "libgz_engine.so")
    if not os.path.lexists(eng):
        os.symlink("../../../galvanise_zero_amd/lib/libgz_engine.so", eng)
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-parameter"]
    objs = []
    procs = []
    tus = ["gz_nn.hip", "runner.hip"] + (sorted(f for f in os.listdir(nn) if f.startswith("trunk_f")) if full else ["trunk_exp.hip"])
    for tu in tus:
        o = os.path.join(work, tu + ".o")
        objs.append(o)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + flags + ["-c", "-o", o, os.path.join(nn, tu)]))
    for p in procs:
        assert p.wait() == 0, name
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + ["-shared", "-o", os.path.join(out, "libgz_nn.so")] + objs +
                          ["-L" + out, "-lgz_engine", "-Wl,-rpath,$ORIGIN"])
    print("built", out)


if __name__ == "__main__":
    names = sys.argv[1:] or ["base"]
    procs = [subprocess.Popen([sys.executable, __file__, "--one", n]) for n in names] if "--one" not in sys.argv else None
    if procs is None:
        build(sys.argv[2])
    else:
        rc = [p.wait() for p in procs]
        sys.exit(max(rc))
