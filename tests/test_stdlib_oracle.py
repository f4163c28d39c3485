"""Pins oracle/stdlib_ref.py (restated libstdc++ std::sort / gamma_distribution<float>, xoroshiro
RNG) against this image's actual libstdc++ via a compiled probe (tests/native/stdlib_probe.cpp)."""
import os
import subprocess

import pytest

from oracle import stdlib_ref as S

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("probe") / "stdlib_probe")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3",
                           os.path.join(HERE, "native", "stdlib_probe.cpp"), "-o", exe])
    return exe


@pytest.mark.parametrize("n,kr,seed", [(5, 2, 1), (16, 3, 2), (17, 2, 3), (40, 4, 4), (90, 3, 5),
                                       (300, 5, 6), (1000, 2, 7), (48, 48, 8)])
def test_std_sort_permutation(probe, n, kr, seed):
    out = subprocess.check_output([probe, "s", str(n), str(kr), str(seed)]).decode().split("\n")
    rows = [tuple(map(int, l.split())) for l in out if l.strip()]
    keys = [r[0] for r in rows]
    expect = [r[1] for r in rows]
    rng = S.Rng(seed)
    pykeys = [rng.getWithMax(kr) for _ in range(n)]
    assert pykeys == keys
    got = S.std_sort(list(range(n)), lambda a, b: keys[a] > keys[b])
    assert got == expect


@pytest.mark.parametrize("alpha,seed", [(0.2256, 1), (0.5, 2), (1.0, 3), (2.7, 4), (0.05, 5)])
def test_gamma_float(probe, alpha, seed):
    n = 200
    out = subprocess.check_output([probe, "g", repr(alpha), str(n), str(seed)]).decode().split()
    expect = [float.fromhex(x) for x in out[:n]]
    last = int(out[n])
    rng = S.Rng(seed)
    g = S.GammaF32(S.F32(alpha))
    got = [float(g(rng)) for _ in range(n)]
    assert got == expect
    assert rng.next_u32() == last
