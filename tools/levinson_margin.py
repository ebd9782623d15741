"""Empirical margin of the reference's Levinson-Durbin on integer PCM.

The OverflowError of `lambda_ ** 2` (encoder.py:476) needs |lambda_| > 1.34e154 and the
floor(log2(inf)) site (encoder.py:503) an infinite coefficient, i.e. |lambda_| overflowing
in the division (encoder.py:469).  For integer PCM the autocorrelation (encoder.py:445-450)
is that of the finite windowed sequence, so the exact reflection coefficients satisfy
|lambda_| < 1; this tool measures how far rounding moves them on adversarial blocks
(near-singular: DC, ramps, low tones, alternating full scale, sparse impulses, 16/24/32-bit,
n = 8..4608, orders up to 32).  The autocorrelation is the oracle's exact restatement
(oracle/flac_oracle.c); the recursion below restates encoder.py:453-479 with the extremes
recorded.  Usage: python tools/levinson_margin.py [trials_per_worker] [workers]
"""
import math
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def lev_extremes(xs):
    order = len(xs) - 1
    coefs = [0.0] * (order + 1)
    coefs[0] = 1.0
    error = xs[0]
    mx, mn_err = 0.0, 1.0
    for k in range(order):
        lam = 0.0
        for j in range(k + 1):
            lam -= coefs[j] * xs[k + 1 - j]
        if error == 0.0:
            return "zero-division", mx, mn_err
        lam /= error
        mx = max(mx, abs(lam))
        if abs(lam) > 1.3e154:
            return "OVERFLOW", mx, mn_err
        for n in range((k + 1) // 2 + 1):
            t = coefs[k + 1 - n] + lam * coefs[n]
            coefs[n] = coefs[n] + lam * coefs[k + 1 - n]
            coefs[k + 1 - n] = t
        error *= 1.0 - lam ** 2
        if xs[0] > 0:
            mn_err = min(mn_err, abs(error) / xs[0])
    return "ok", mx, mn_err


def block(rnd):
    n = rnd.choice([8, 9, 12, 16, 24, 32, 64, 128, 192, 576, 1152, 4608])
    bits = rnd.choice([16, 16, 24, 32])
    A = rnd.choice([1, 3, 100, (1 << (bits - 1)) - 1])
    kind = rnd.randrange(8)
    if kind == 0:
        xs = [rnd.randint(-A, A) for _ in range(n)]
    elif kind == 1:
        c = rnd.randint(-A, A)
        xs = [c + rnd.choice([0, 0, 0, 1, -1]) for _ in range(n)]
    elif kind == 2:
        xs = [A if i % 2 else -A for i in range(n)]
    elif kind == 3:
        d = rnd.randint(1, 5)
        xs = [round(A * (i / n) ** d) for i in range(n)]
    elif kind == 4:
        f = 10.0 ** rnd.uniform(-4, -0.3)
        ph = rnd.random() * 6.3
        xs = [round(A * math.sin(2 * math.pi * f * i + ph)) for i in range(n)]
    elif kind == 5:
        xs = [0] * n
        for _ in range(rnd.randint(1, 3)):
            xs[rnd.randrange(n)] = rnd.randint(-A, A)
    elif kind == 6:
        xs = [rnd.choice([-A, A, 0]) for _ in range(n)]
    else:
        g = 1.0 + 10.0 ** rnd.uniform(-6, -1)
        xs = [round(A * g ** (i - n)) for i in range(n)]
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    return [max(lo, min(hi, x)) for x in xs]


def work(args):
    seed, trials = args
    import oracle
    import numpy as np
    rnd = random.Random(seed)
    worst = (0.0, None)
    min_err = 1.0
    outcomes = {}
    for _ in range(trials):
        xs = block(rnd)
        n = len(xs)
        _, w = oracle.tukey(n)
        win = np.asarray(xs, dtype=np.float64) * np.asarray(w)
        L = min(n - 1, rnd.choice([8, 12, 32]))
        ac = [oracle.autocorrelation(win, lag) for lag in range(L + 1)]
        r, mx, me = lev_extremes(ac)
        outcomes[r] = outcomes.get(r, 0) + 1
        if r == "ok":
            min_err = min(min_err, me)
        if mx > worst[0]:
            worst = (mx, (n, L, xs[:8]))
    return worst, min_err, outcomes


def main():
    import multiprocessing as mp
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    with mp.Pool(workers) as p:
        res = p.map(work, [(s, trials) for s in range(workers * 4)])
    total = {}
    for _, _, o in res:
        for k, v in o.items():
            total[k] = total.get(k, 0) + v
    worst = max(res, key=lambda r: r[0][0])[0]
    print("blocks:", sum(total.values()), "outcomes:", total)
    print("max |lambda_|: %.6f  (block n=%d L=%d head=%s)" % (worst[0], *worst[1]))
    print("min |error|/acf[0] over blocks without an exception: %.3e" % min(r[1] for r in res))


if __name__ == "__main__":
    main()
