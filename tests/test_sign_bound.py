"""CPU soundness check of the sign-correlation bound the int8-MFMA path prunes with
(k_resid.h mf8_candidate_sums): on units of every kind (config-3 synthetic
24-bit, tones, AR(1), white and small noise, 16-bit shapes) the bound of every LPC order is
at most that order's exact sum(|r|) from the oracle, and a unit it decides has its best LPC
sum strictly above its best fixed sum (encoder.py:133-157: no LPC win, no tie)."""
import numpy as np
import pytest

import oracle
import sign_bound


def _units(n, bits, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    top = 2 ** (bits - 1) - 1
    rows = [oracle.synth_batch(0, 8, n, bits, seed, dtype=np.int32)]
    x = []
    for u in range(4):
        x.append(0.6 * top * np.sin(2 * np.pi * (u + 1) * 441 / n * t) + rng.normal(0, 0.01 * top * u, n))
    for u in range(4):
        w = rng.normal(0, top / 40, n)
        a = w.copy()
        a[1:] += (0.95 if u % 2 else -0.6) * w[:-1]
        x.append(a)
    x.append(rng.normal(0, top / 8, n))
    x.append(rng.normal(0, 3, n))
    rows.append(np.clip(np.round(np.array(x)), -top - 1, top).astype(np.int32))
    return np.ascontiguousarray(np.concatenate(rows))


@pytest.mark.parametrize("n,bits,L,q,lmax", [(4096, 24, 32, 15, 32), (16384, 24, 32, 12, 32), (4608, 16, 32, 15, 32),
                                             (4608, 16, 12, 5, 16), (4608, 16, 12, 9, 16)])
def test_sign_bound_is_a_lower_bound(n, bits, L, q, lmax):
    """lmax 16: k_resid's 16-bit paths at L <= 12 take R' = [16, n) (k_resid.h sb16_chunk)."""
    a = _units(n, bits, n + q)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 8 if n % 256 == 0 else 5), n,
                               sample_bits=bits, threads=8)
    decided = 0
    for u in range(len(a)):
        if int(ora["meta"]["status"][u]) != 0 or int(ora["lpc_records"][u][0]) != 0:
            continue
        rec, fs, ls = ora["lpc_records"][u], ora["fixed_sums"][u], ora["lpc_sums"][u]
        for hi in (None, n // 2, 4096):  # the whole R, and k_resid_sb's first tests ([lmax, hi))
            for p, lb in enumerate(sign_bound.order_bounds(a[u], rec, L, lmax=lmax, hi=hi), start=1):
                if lb is not None:
                    assert lb <= int(ls[p - 1]), (u, p, hi, lb, int(ls[p - 1]))
        if sign_bound.decides(a[u], rec, L, fs, lmax=lmax, split_end=n // 2):
            decided += 1
            assert int(ora["meta"]["lpc_sum"][u]) > int(ora["meta"]["fixed_sum"][u]), u
    assert decided > 0
