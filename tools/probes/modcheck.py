"""CPU check of the encode's residue forms against exact integer residues: x reduced modulo a
group product P in f64, then 1 (pairs) or 2 (triples) f32 steps per modulus, for |x| up to 2^L
(split.hip ModGroups).  Prints the mismatch count per magnitude and form."""
import numpy as np, sys
P = [256,255,253,251,247,241,239,233,229,227,223,217,211,199,197,193,191,181,179,173]
def f32_step(t, p):
    rf = np.float32(1.0)/np.float32(p)
    y = (t*rf).astype(np.float32)
    y = np.rint(y).astype(np.float32)
    return (t + y*np.float32(-p)).astype(np.float32)  # fma exact for these magnitudes? emulate via f64
def f32_step_fma(t, p):
    rf = np.float32(np.float32(1.0)/np.float32(p))
    y = np.rint((t.astype(np.float32)*rf).astype(np.float32))
    r = t.astype(np.float64) + y.astype(np.float64)*(-p)   # fma: exact product+sum, single rounding to f32
    return r.astype(np.float32)
def scheme(a, N, g, steps):
    out = {}
    j = 0
    while j < N:
        grp = P[j:j+g]; Pp = float(np.prod(grp))
        rP = 1.0/Pp
        q = np.rint(a*rP)
        # fma(q, -P, a) exact-rounded in f64: compute with python ints for exactness of single rounding
        t = np.array([float(int(ai) - int(qi)*int(Pp)) for ai, qi in zip(a, q)])
        t32 = t.astype(np.float32)
        for p in grp:
            r = t32
            for _ in range(steps): r = f32_step_fma(r, p)
            out[p] = r.astype(np.int64)
        j += g
    return out
rng = np.random.default_rng(1)
for L in [53, 58, 60, 66, 70, 72, 73, 74, 76]:
    a = np.ldexp(rng.random(20000)*2-1, L)
    a = np.trunc(a)
    ai = [int(x) for x in a]
    for g, steps in [(3, 2), (2, 1)]:
        res = scheme(a, 20, g, steps)
        bad = 0
        for p in P:
            exp = np.array([((x + p//2) % p) - p//2 for x in ai])  # symmetric residue in [-p/2, p/2)
            got = res[p]
            if p == 256:
                bad += np.sum((got & 255) != (exp & 255))
            else:
                bad += np.sum(got != exp)
        print(f"L={L} groups={g} steps={steps}: mismatches {bad}")

# f32 operands: mod_8i<float>'s four f32 steps from x itself vs exact, for float-valued |x| < 2^L
def f32_four_steps(x, p):
    t = x.astype(np.float32)
    for _ in range(4):
        t = f32_step_fma(t, p)
    return t.astype(np.int64)
for L in [40, 44, 45, 46, 47, 48, 50]:
    x = np.trunc(np.ldexp((rng.random(20000) * 2 - 1).astype(np.float32).astype(np.float64), L)).astype(np.float32)
    xi = [int(v) for v in x.astype(np.float64)]
    bad = 0
    for p in P:
        exp = np.array([((v + p // 2) % p) - p // 2 for v in xi])
        got = f32_four_steps(x, p)
        bad += np.sum((got & 255) != (exp & 255)) if p == 256 else np.sum(got != exp)
    print(f"f32 four steps, L={L}: mismatches {bad}")
