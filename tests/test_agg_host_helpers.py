"""Host helpers of the Aggregate C-ABI (no GPU): the exact limb sum is rounded once to the nearest double, and the
order-preserving words decode to the value bits (include/hyrise_amd.h, hy_agg_float_sum / hy_agg_decode_ordered)."""
import ctypes
import math
import random
import struct
from fractions import Fraction

import pytest


def float_sum(hy, limbs, emin, special=0):
    arr = (ctypes.c_uint64 * max(1, len(limbs)))(*[v & (2**64 - 1) for v in limbs])
    out = ctypes.c_double()
    hy.capi.check(hy.capi.lib.hy_agg_float_sum(arr, len(limbs), emin, special, ctypes.byref(out)), "float_sum")
    return out.value


def exact(limbs, emin):
    return sum(Fraction(v) * Fraction(2) ** (32 * i + emin) for i, v in enumerate(limbs))


@pytest.mark.parametrize("seed", range(20))
def test_float_sum_is_correctly_rounded(hy, seed):
    rng = random.Random(seed)
    n = rng.choice([9, 66])
    emin = -149 if n == 9 else -1074
    limbs = [0] * n
    lo = rng.randrange(0, n - 2)
    for i in range(lo, min(n, lo + rng.randrange(1, 5))):
        limbs[i] = rng.randrange(-(2**62), 2**62)
    got = float_sum(hy, limbs, emin)
    want = float(exact(limbs, emin))
    assert got == want, (limbs, got, want)


def test_float_sum_of_float_values_matches_fsum(hy):
    rng = random.Random(7)
    vals = [struct.unpack("f", struct.pack("f", rng.uniform(-1e6, 1e6)))[0] for _ in range(1000)]
    limbs = [0] * 9
    for v in vals:  # the device's decomposition, restated: m * 2^(e-150) split into 32-bit pieces at shift e-1
        b = struct.unpack("I", struct.pack("f", v))[0]
        e, m, neg = (b >> 23) & 0xFF, b & 0x7FFFFF, b >> 31
        if e == 0 and m == 0:
            continue
        if e:
            m |= 0x800000
        shift = e - 1 if e else 0
        c = m << (shift & 31)
        for k in range(2):
            p = (c >> (32 * k)) & 0xFFFFFFFF
            limbs[(shift >> 5) + k] += -p if neg else p
    assert float_sum(hy, limbs, -149) == math.fsum(vals)


def test_float_sum_specials(hy):
    assert float_sum(hy, [0] * 9, -149, 1) == math.inf
    assert float_sum(hy, [0] * 9, -149, 2) == -math.inf
    assert math.isnan(float_sum(hy, [0] * 9, -149, 3))
    assert math.isnan(float_sum(hy, [0] * 9, -149, 4))
    assert float_sum(hy, [0] * 9, -149, 0) == 0.0


@pytest.mark.parametrize("type_,values", [
    (1, [-2**31, -5, -1, 0, 1, 7, 2**31 - 1]),
    (2, [-2**63, -9, 0, 3, 2**63 - 1]),
    (3, [-math.inf, -1e30, -1.5, -0.0, 0.0, 1e-40, 2.5, math.inf]),
    (4, [-math.inf, -1e300, -1.5, 0.0, 5e-324, 2.5, 1e300]),
])
def test_ordered_words_round_trip_and_preserve_order(hy, type_, values):
    def bits(v):
        if type_ == 1:
            return v & 0xFFFFFFFF
        if type_ == 2:
            return v & (2**64 - 1)
        if type_ == 3:
            return struct.unpack("I", struct.pack("f", v))[0]
        return struct.unpack("Q", struct.pack("d", v))[0]

    def ordered(b):  # device ordered_bits(), restated
        if type_ == 1:
            return b ^ 0x80000000
        if type_ == 2:
            return b ^ (1 << 63)
        if type_ == 3:
            return (~b & 0xFFFFFFFF) if b >> 31 else b | 0x80000000
        return (~b & (2**64 - 1)) if b >> 63 else b | (1 << 63)

    words = [ordered(bits(v)) for v in values]
    assert words == sorted(words)
    for v, w in zip(values, words):
        assert hy.capi.lib.hy_agg_decode_ordered(w, type_) == bits(v)
