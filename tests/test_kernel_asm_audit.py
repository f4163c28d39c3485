"""The split kernels' inline-asm MFMA chains are hazard-free as compiled (tests/kernel_asm_audit.py):
the auditor itself on synthetic assembly, then the gfx950 assembly of every trunk kernel that runs
chains (hipcc -S of one translation unit instantiating them, CPU only; the F = 64 and 256 split
kernels run the unrolled conv with builtins)."""
import os
import shutil
import subprocess

import pytest

import kernel_asm_audit as kaa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NN = os.path.join(ROOT, "galvanise_zero_amd", "csrc", "nn")
HIPCC = "/opt/rocm/bin/hipcc"

CHAIN = """\t;;#ASMSTART
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[10:13], v[20:23], a[0:3]
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[10:13], v[24:27], a[0:3]
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[14:17], v[20:23], a[0:3]
\t;;#ASMEND
"""


def kernel(body):
    return "_ZN4gznn4testEv:\n" + body + ".Lfunc_end0:\n"


def violations(body):
    (n, bad), = kaa.audit(kernel(body)).values()
    assert n == 3
    return bad


def test_auditor_clean_chain():
    body = ("\tds_read_b128 v[20:23], v1\n\tglobal_load_dwordx4 v[10:13], v2, s[0:1]\n\ts_waitcnt vmcnt(0)\n" + CHAIN +
            "\t;;#ASMSTART\n\ts_nop 15\n\ts_nop 7\n\t;;#ASMEND\n\tv_accvgpr_read_b32 v30, a0\n")
    assert violations(body) == []


def test_auditor_rule1_operand_write():
    assert any("rule 1" in v for v in violations("\tv_mov_b32 v21, v5\n" + CHAIN))
    assert any("rule 1" in v for v in violations("\tv_accvgpr_write_b32 a2, 0\n" + CHAIN))
    # two states of padding in between: fine
    assert violations("\tv_mov_b32 v21, v5\n\ts_nop 1\n" + CHAIN) == []


def test_auditor_rule2_early_read():
    assert any("rule 2" in v for v in violations(CHAIN + "\ts_nop 7\n\tv_accvgpr_read_b32 v30, a1\n"))
    assert violations(CHAIN + "\ts_nop 15\n\ts_nop 7\n\tv_accvgpr_read_b32 v30, a1\n") == []


def test_auditor_rule3_loop_copy():
    # an operand written at the end of an iteration, read by the chain opening the next one
    body = (".LBB0_1:\n" + CHAIN + "\ts_nop 15\n\ts_nop 7\n\tv_mov_b32 v10, v40\n"
            "\ts_cbranch_scc1 .LBB0_1\n")
    assert any("rule 1" in v for v in violations(body))
    body = (".LBB0_1:\n\tv_accvgpr_mov_b32 a5, a1\n\ts_nop 15\n\ts_nop 7\n" + CHAIN + "\ts_nop 15\n\ts_nop 7\n"
            "\ts_cbranch_scc1 .LBB0_1\n")
    assert any("rule 3" in v for v in violations(body))


# every trunk instantiation that runs the split looped conv (the F = 128 split kernels, v1 and v2,
# one and two boards, the two-group, the 8-wave and the two-groups-of-two kernels), in one
# translation unit (compiled with the library's flags)
AUDIT_TU = """#include "trunk_variants.h"
namespace gznn {
template __global__ void trunk_kernel<128, 2, 1, 1, 3>(KParams);
template __global__ void trunk_kernel<128, 2, 2, 1, 3>(KParams);
template __global__ void trunk_kernel<128, 3, 1, 1, 3>(KParams);
template __global__ void trunk_kernel<128, 3, 2, 1, 3>(KParams);
template __global__ void trunk_kernel<128, 4, 1, 1, 3>(KParams);
template __global__ void trunk_kernel<128, 4, 2, 1, 3>(KParams);
template __global__ void trunk_kernel_v2<128, 4, 1, 1, 3>(KParams);
template __global__ void trunk_kernel_v2<128, 4, 2, 1, 3>(KParams);
template __global__ void trunk_kernel8<128, 4, 3>(KParams);
template __global__ void trunk_kernel_w8<128, 2, 3>(KParams);
template __global__ void trunk_kernel_w8<128, 3, 3>(KParams);
template __global__ void trunk_kernel_w8<128, 4, 3>(KParams);
template __global__ void trunk_kernel_h2<128, 2, 3>(KParams);
template __global__ void trunk_kernel_h2<128, 4, 3>(KParams);
}
"""


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="hipcc absent")
def test_compiled_chains_hazard_free(tmp_path):
    src = tmp_path / "audit_tu.hip"
    src.write_text(AUDIT_TU)
    out = tmp_path / "audit_tu.s"
    subprocess.check_call([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-parameter",
                           "-ffp-contract=on", "--cuda-device-only", "-S", "-I", NN, "-o", str(out), str(src)],
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    res = kaa.audit(out.read_text())
    assert len(res) == 14, sorted(res)    # every instantiation above runs chains
    for name, (n, bad) in res.items():
        assert n > 0
        assert bad == [], (name, bad[:5])
    assert any("ILi128ELi4ELi2ELi1ELi3E" in k for k in res)   # the round-4 headline kernel
    assert any("trunk_kernel_h2ILi128ELi4ELi3E" in k for k in res)   # the headline kernel
