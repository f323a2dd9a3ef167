"""The uint8 transform's division by reciprocal + one fma correction is bit-identical to the IEEE
division on every operand a uint8 image can produce (csrc/layers.hip div_fast / u8_fast_div).

The device takes that path only when the launcher's host check (the same enumeration, in C++) passes
for the actual mean / std; this test restates the enumeration with exact rational arithmetic for
GeneralizedRCNNTransform's ImageNet constants (reference detect.py:24,30 -> torchvision defaults), so
the claim does not rest on the host's own fmaf alone."""
from fractions import Fraction

import numpy as np

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def rn32(q):
    """Round the rational q to the nearest float32, ties to even."""
    f = np.float32(float(q))
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        d = abs(Fraction(float(c)) - q)
        key = (d, int(np.float32(c).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, np.float32(c))
    return best[1]


def fma(a, b, c):
    return rn32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def div_fast(a, b, rb):
    q = np.float32(a * rb)
    return fma(fma(-q, b, a), rb, q)


def test_div_fast_matches_ieee_division_on_every_uint8_operand():
    r255 = np.float32(1) / np.float32(255)
    plain_mul_differs = 0
    for x in range(256):
        xf = np.float32(x)
        t = np.float32(xf / np.float32(255))
        assert div_fast(xf, np.float32(255), r255) == t, x
        plain_mul_differs += np.float32(xf * r255) != t
        for m, s in zip(MEAN, STD):
            m, s = np.float32(m), np.float32(s)
            a = np.float32(t - m)
            assert div_fast(a, s, np.float32(1) / s) == np.float32(a / s), (x, m, s)
    assert plain_mul_differs > 0  # the correction step is needed: a bare reciprocal multiply is not exact
