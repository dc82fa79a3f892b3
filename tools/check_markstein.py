"""CPU check of the branch-free int8 quantiser division (csrc/common.h q8_exact).

    python tools/check_markstein.py [n_search]

q0 = fl(v * y) with y = fl(1/s) can be up to ~1.5 ulp from v/s, which is outside Markstein's
precondition (a FAITHFUL q), so ONE correction fl(q0 + fl(v - s q0) y) is not guaranteed to be
fl(v / s).  After that first correction q1 is within ~0.5 ulp + 2^-23 ulp (faithful), so a SECOND
correction q2 = fl(q1 + (v - s q1) y), whose remainder is exact, is fl(v / s) by Markstein's theorem
(y within half an ulp of 1/s, q1 faithful, round to nearest; no overflow / subnormal quotients in
the quantiser's range).  This script
  1. searches adversarially (vectorised, float64-exact intermediates) for operands where the
     one-step form differs from fl(v / s) -- scales with all-ones mantissas, quotients at the top of
     a binade, v near half-integer multiples of s;
  2. re-checks every hit, plus random and +-2-ulp-around-tie operands, with EXACT rational
     arithmetic (fractions.Fraction, single rounding to float32 -- no float64 double rounding)
     for both forms, and fails if the two-step form ever differs.
"""
import sys
from fractions import Fraction

import numpy as np

f32 = np.float32


def rn32(fr: Fraction) -> np.float32:
    """Round an exact rational to float32, round-half-even, one rounding (normal range)."""
    if fr == 0:
        return f32(0.0)
    sign = -1 if fr < 0 else 1
    a = abs(fr)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    ulp = Fraction(2) ** (max(e, -126) - 23)
    return f32(sign * float(round(a / ulp) * ulp))


def fma32(a, b, c):
    return rn32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def one_step(v, s, y):
    q = f32(v * y)
    return fma32(fma32(-q, s, v), y, q)


def two_step(v, s, y):
    q1 = one_step(v, s, y)
    return fma32(fma32(-q1, s, v), y, q1)


def exact(v, s):
    return rn32(Fraction(float(v)) / Fraction(float(s)))


def search(n, rng):
    """Vectorised hunt for one-step failures (float64 holds the products exactly)."""
    hits = []
    for mode in range(3):
        if mode == 0:   # scales with (nearly) all-ones mantissas
            s = (2.0 - rng.integers(1, 64, n) * 2.0 ** -23) * 2.0 ** rng.integers(-14, 4, n)
        elif mode == 1:
            s = np.exp(rng.uniform(-12, 3, n))
        else:           # mantissa near 1 (reciprocal near the top of its binade)
            s = (1.0 + rng.integers(0, 64, n) * 2.0 ** -23) * 2.0 ** rng.integers(-14, 4, n)
        s = s.astype(np.float32)
        k = rng.integers(-128, 128, n).astype(np.float64)
        # quotient near k + 0.5 or near the top of a binade
        tgt = np.where(rng.random(n) < 0.5, k + 0.5, (2.0 - rng.random(n) * 2.0 ** -20) * 2.0 ** rng.integers(-8, 7, n))
        v = (tgt * s.astype(np.float64)).astype(np.float32)
        v = np.nextafter(v, np.where(rng.random(n) < 0.5, np.inf, -np.inf).astype(np.float32)) \
            if mode else v
        y = (np.float32(1.0) / s).astype(np.float32)
        vd, sd, yd = v.astype(np.float64), s.astype(np.float64), y.astype(np.float64)
        q0 = (v * y).astype(np.float32)
        e0 = (vd - q0.astype(np.float64) * sd).astype(np.float32)          # exact in f64, one rounding
        q1 = (q0.astype(np.float64) + e0.astype(np.float64) * yd).astype(np.float32)
        ex = (vd / sd).astype(np.float32)                                   # f64 quotient: no double-rounding hit
        bad = np.nonzero(q1 != ex)[0]
        hits += [(v[i], s[i]) for i in bad[:200]]
    return hits


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    rng = np.random.default_rng(0)
    cand = search(n, rng)
    one_bad = two_bad = checked = 0
    cases = list(cand)
    for _ in range(4000):   # random operands
        s = f32(np.exp(rng.uniform(-12, 3)))
        cases.append((f32(rng.normal() * float(s) * rng.uniform(0, 200)), s))
    for _ in range(4000):   # +-2 ulp around ties
        s = f32(np.exp(rng.uniform(-12, 3)))
        v = f32((int(rng.integers(-130, 130)) + 0.5) * float(s))
        for d in (-2, -1, 0, 1, 2):
            vv = v
            for _ in range(abs(d)):
                vv = np.nextafter(vv, f32(np.inf) if d > 0 else f32(-np.inf), dtype=np.float32)
            cases.append((vv, s))
    for v, s in cases:
        y = f32(f32(1.0) / s)
        ex = exact(v, s)
        checked += 1
        if one_step(v, s, y) != ex:
            one_bad += 1
        if two_step(v, s, y) != ex:
            two_bad += 1
            if two_bad < 10:
                print("TWO-STEP MISMATCH", v, s)
    print(f"search candidates {len(cand)}; exact checks {checked}: one-step mismatches {one_bad}, "
          f"two-step mismatches {two_bad}")
    sys.exit(1 if two_bad else 0)


if __name__ == "__main__":
    main()
