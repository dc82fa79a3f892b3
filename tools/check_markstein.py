"""CPU check of the branch-free int8 quantiser division (csrc/common.h q8_exact): q = fl(v * fl(1/s)),
one Markstein correction fl(q + fl(v - s q) fl(1/s)) == fl(v / s), against exact rational
division (fractions.Fraction) on random and near-tie operands.  python tools/check_markstein.py"""
import numpy as np
from fractions import Fraction
rng = np.random.default_rng(0)
f32 = np.float32
def fma32(a, b, c):
    # exact a*b + c rounded once to float32 (via Fraction)
    return f32(float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))))
def rn32(x): return f32(x)
bad = 0; n = 0
def check(v, s):
    global bad, n
    inv = f32(f32(1.0) / s)
    q = f32(v * inv)
    e = fma32(-q, s, v)
    q2 = fma32(e, inv, q)
    exact = f32(float(Fraction(float(v)) / Fraction(float(s))))
    n += 1
    if q2 != exact:
        bad += 1
        if bad < 10: print("mismatch", v, s, q2, exact)
# random
for _ in range(20000):
    s = f32(np.exp(rng.uniform(-12, 3)))
    v = f32(rng.normal() * float(s) * rng.uniform(0, 200))
    check(v, s)
# near-ties: v = (k + 0.5) * s perturbed by few ulps
for _ in range(20000):
    s = f32(np.exp(rng.uniform(-12, 3)))
    k = rng.integers(-130, 130)
    v = f32((k + 0.5) * float(s))
    for d in (-2, -1, 0, 1, 2):
        vv = np.nextafter(v, f32(np.inf) if d > 0 else f32(-np.inf), dtype=np.float32) if d else v
        if abs(d) == 2: vv = np.nextafter(vv, f32(np.inf) if d > 0 else f32(-np.inf), dtype=np.float32)
        check(vv, s)
print("checked", n, "mismatches", bad)
