"""ORACLE (test infrastructure only) -- restatements of the C/C++ runtime pieces the reference's
PUCT code relies on, so oracle/puct_ref.py reproduces results bit for bit.

Third-party algorithms restated here (absent from /root/reference; versions = this image's
toolchain, which the native engine is also built with):
  * libstdc++ 11 std::sort (introsort + final insertion sort, bits/stl_algo.h / stl_heap.h): the
    reference sorts children with std::sort and unstable tie order decides PUCT argmax ties
    (evaluator.cpp:242-263, node.cpp:316-373).
  * libstdc++ 11 std::gamma_distribution<float> / normal_distribution<float> /
    generate_canonical<float,24> (bits/random.tcc, random.h): Dirichlet noise (evaluator.cpp:1249).
  * glibc libm logf / powf / pow via ctypes (the engine calls the same functions).
  * xoroshiro128+ (Blackman & Vigna) with splitmix64 seeding: the engine's replacement for the
    unseeded K273::xoroshiro128plus32 (galvanise_zero_amd/csrc/engine/rng.h).
Pinned by tests/test_stdlib_oracle.py against probes compiled from this image's libstdc++.
"""
import ctypes
import ctypes.util
import math

import numpy as np

F32 = np.float32
M64 = (1 << 64) - 1

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]
_libm.powf.restype = ctypes.c_float
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
_libm.sqrtf.restype = ctypes.c_float
_libm.sqrtf.argtypes = [ctypes.c_float]
_libm.pow.restype = ctypes.c_double
_libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]
_libm.nextafterf.restype = ctypes.c_float
_libm.nextafterf.argtypes = [ctypes.c_float, ctypes.c_float]


def logf(x):
    return F32(_libm.logf(float(x)))


def powf(x, y):
    return F32(_libm.powf(float(x), float(y)))


def sqrtf(x):
    return F32(_libm.sqrtf(float(x)))


def pow_d(x, y):
    return _libm.pow(float(x), float(y))


# ---- RNG (csrc/engine/rng.h) -------------------------------------------------------------------

def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return state, z ^ (z >> 31)


def rng_mix(global_seed, game_index, stream):
    x = (global_seed ^ ((game_index * 0xD1B54A32D192ED03) & M64) ^ ((stream * 0x8CB92BA72F3D8DD7) & M64)) & M64
    _, z = splitmix64(x)
    return z


def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


class Rng(object):
    def __init__(self, seed=0x853c49e6748fea9b):
        self.seed(seed)

    def seed(self, seed):
        x, self.s0 = splitmix64(seed & M64)
        x, self.s1 = splitmix64(x)
        if self.s0 == 0 and self.s1 == 0:
            self.s1 = 1

    def next_u32(self):
        a, b = self.s0, self.s1
        result = (a + b) & M64
        b ^= a
        self.s0 = _rotl(a, 24) ^ b ^ ((b << 16) & M64)
        self.s1 = _rotl(b, 37)
        return result >> 32

    def get(self):
        return self.next_u32() * (1.0 / 4294967296.0)

    def getWithMax(self, upper):
        return self.next_u32() % upper if upper else 0


# ---- libstdc++ std::sort -------------------------------------------------------------------------

_THRESHOLD = 16


def _lg(n):
    return n.bit_length() - 1


def std_sort(a, less):
    """In-place std::sort(a.begin(), a.end(), less) with libstdc++ 11's exact element moves."""
    n = len(a)
    if n == 0:
        return a
    _introsort_loop(a, 0, n, _lg(n) * 2, less)
    _final_insertion_sort(a, 0, n, less)
    return a


def _move_median_to_first(a, result, x, y, z, less):
    if less(a[x], a[y]):
        if less(a[y], a[z]):
            a[result], a[y] = a[y], a[result]
        elif less(a[x], a[z]):
            a[result], a[z] = a[z], a[result]
        else:
            a[result], a[x] = a[x], a[result]
    elif less(a[x], a[z]):
        a[result], a[x] = a[x], a[result]
    elif less(a[y], a[z]):
        a[result], a[z] = a[z], a[result]
    else:
        a[result], a[y] = a[y], a[result]


def _unguarded_partition(a, first, last, pivot, less):
    while True:
        while less(a[first], a[pivot]):
            first += 1
        last -= 1
        while less(a[pivot], a[last]):
            last -= 1
        if not (first < last):
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _introsort_loop(a, first, last, depth_limit, less):
    while last - first > _THRESHOLD:
        if depth_limit == 0:
            _heap_select(a, first, last, last, less)
            _sort_heap(a, first, last, less)
            return
        depth_limit -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(a, first, first + 1, mid, last - 1, less)
        cut = _unguarded_partition(a, first + 1, last, first, less)
        _introsort_loop(a, cut, last, depth_limit, less)
        last = cut


def _unguarded_linear_insert(a, last, less):
    val = a[last]
    nxt = last - 1
    while less(val, a[nxt]):
        a[last] = a[nxt]
        last = nxt
        nxt -= 1
    a[last] = val


def _insertion_sort(a, first, last, less):
    if first == last:
        return
    for i in range(first + 1, last):
        if less(a[i], a[first]):
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            _unguarded_linear_insert(a, i, less)


def _final_insertion_sort(a, first, last, less):
    if last - first > _THRESHOLD:
        _insertion_sort(a, first, first + _THRESHOLD, less)
        for i in range(first + _THRESHOLD, last):
            _unguarded_linear_insert(a, i, less)
    else:
        _insertion_sort(a, first, last, less)


def _push_heap(a, first, hole, top, value, less):
    parent = (hole - 1) // 2
    while hole > top and less(a[first + parent], value):
        a[first + hole] = a[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[first + hole] = value


def _adjust_heap(a, first, hole, length, value, less):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if less(a[first + second], a[first + second - 1]):
            second -= 1
        a[first + hole] = a[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        a[first + hole] = a[first + second - 1]
        hole = second - 1
    _push_heap(a, first, hole, top, value, less)


def _make_heap(a, first, last, less):
    length = last - first
    if length < 2:
        return
    parent = (length - 2) // 2
    while True:
        _adjust_heap(a, first, parent, length, a[first + parent], less)
        if parent == 0:
            return
        parent -= 1


def _pop_heap(a, first, last, result, less):
    value = a[result]
    a[result] = a[first]
    _adjust_heap(a, first, 0, last - first, value, less)


def _heap_select(a, first, middle, last, less):
    _make_heap(a, first, middle, less)
    for i in range(middle, last):
        if less(a[i], a[first]):
            _pop_heap(a, first, middle, i, less)


def _sort_heap(a, first, last, less):
    while last - first > 1:
        last -= 1
        _pop_heap(a, first, last, last, less)


# ---- libstdc++ gamma_distribution<float> --------------------------------------------------------

def generate_canonical_f32(rng):
    """generate_canonical<float, 24>(urng) for a 32-bit URBG: one draw."""
    s = F32(rng.next_u32()) * F32(1.0)
    tmp = F32(4294967296.0)
    ret = F32(s / tmp)
    if ret >= F32(1.0):
        ret = F32(_libm.nextafterf(1.0, 0.0))
    return ret


class NormalF32(object):
    """normal_distribution<float>(0, 1) (Marsaglia polar method with one cached value)."""

    def __init__(self):
        self.saved = None

    def __call__(self, rng):
        if self.saved is not None:
            ret, self.saved = self.saved, None
        else:
            while True:
                x = F32(float(F32(2.0) * generate_canonical_f32(rng)) - 1.0)
                y = F32(float(F32(2.0) * generate_canonical_f32(rng)) - 1.0)
                r2 = F32(F32(x * x) + F32(y * y))
                if not (float(r2) > 1.0 or float(r2) == 0.0):
                    break
            mult = sqrtf(F32(F32(F32(-2) * logf(r2)) / r2))
            self.saved = F32(x * mult)
            ret = F32(y * mult)
        return F32(F32(ret * F32(1.0)) + F32(0.0))


class GammaF32(object):
    """gamma_distribution<float>(alpha, 1) (Marsaglia & Tsang)."""

    def __init__(self, alpha, beta=1.0):
        self.alpha = F32(alpha)
        self.beta = F32(beta)
        self.malpha = F32(self.alpha + F32(1.0)) if float(self.alpha) < 1.0 else self.alpha
        a1 = F32(self.malpha - F32(F32(1.0) / F32(3.0)))
        self.a2 = F32(F32(1.0) / sqrtf(F32(F32(9.0) * a1)))
        self.nd = NormalF32()

    def __call__(self, rng):
        a1 = F32(self.malpha - F32(F32(1.0) / F32(3.0)))
        while True:
            while True:
                n = self.nd(rng)
                v = F32(F32(1.0) + F32(self.a2 * n))
                if not (float(v) <= 0.0):
                    break
            v = F32(F32(v * v) * v)
            u = generate_canonical_f32(rng)
            nd = float(n)
            c1 = float(u) > float(F32(1.0)) - 0.0331 * nd * nd * nd * nd
            if not c1:
                break
            rhs = 0.5 * nd * nd + float(a1) * (1.0 - float(v) + float(logf(v)))
            if not (float(logf(u)) > rhs):
                break
        if self.alpha == self.malpha:
            return F32(F32(a1 * v) * self.beta)
        while True:
            u = generate_canonical_f32(rng)
            if float(u) != 0.0:
                break
        return F32(F32(F32(powf(u, F32(F32(1.0) / self.alpha)) * a1) * v) * self.beta)


def f32_from_double(x):
    return F32(x)


def isclose_ulp(a, b):
    return a == b or (math.isnan(a) and math.isnan(b))
