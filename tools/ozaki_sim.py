# Accuracy of an Ozaki-style int8 digit emulation of one fp64 Gram entry:
# balanced base-128 digits of x * 2^(7s-2), the s(s+1)/2 digit products summed exactly, against
# the fp64 sum and an extended-precision reference.  Usage: python tools/ozaki_sim.py
import numpy as np, math
rng = np.random.default_rng(1)
n = 1_000_000
def vec(local):
    v = rng.standard_normal(n)
    if local:
        v *= 1e-3
        v[rng.integers(0, n, 5)] += rng.standard_normal(5)
    return v / np.linalg.norm(v)
def digits(x, s, sc):
    v = np.round(x * 2.0**sc).astype(np.int64)
    d = [None] * s
    for p in range(s - 1, 0, -1):   # balanced digits from the bottom
        dp = ((v + 64) & 127) - 64
        d[p] = dp
        v = (v - dp) >> 7
    d[0] = v
    assert (d[0] >= -128).all() and (d[0] <= 127).all(), (d[0].min(), d[0].max())
    return d
def ozaki_dot(x, y, s, extra=0):
    sc = 7 * s - 2
    dx = digits(x, s, sc); dy = digits(y, s, sc)
    tot = 0.0
    for dd in range(0, s + extra):
        acc = 0
        for p in range(max(0, dd - s + 1), min(dd, s - 1) + 1):
            acc += int(np.dot(dx[p], dy[dd - p]))
        tot += acc * 2.0**(7*(2*(s-1)-dd))
    return tot / 2.0**(2*sc)
for local in (False, True):
    x, y = vec(local), vec(local)
    y = y - (x @ y) * x + 1e-9 * x
    exact = math.fsum((x.astype(np.longdouble) * y.astype(np.longdouble)).tolist())
    f64 = float(x @ y)
    for s in (6, 7, 8):
        oz = ozaki_dot(x, y, s)
        print(f"local={local} s={s} pairs={s*(s+1)//2}: |fp64-exact| {abs(f64-exact):.2e}  |ozaki-exact| {abs(oz-exact):.2e}")
