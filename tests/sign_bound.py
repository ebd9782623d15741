"""Restatement of the int8-MFMA path's sign-correlation bound (flac-py_amd/csrc/k_resid.h,
mf8_candidate_sums) on the oracle's LPC record, shared by the CPU soundness test and the GPU
tier test.  Test infrastructure only."""
import numpy as np


def order_bounds(x, rec, L, lmax=32, hi=None):
    """Per LPC order p = 1..L: the kernel's integer lower bound of sum|r| (r: the reference's
    residual of order p, encoder.py:537-548), or None for a coefficient-less order ((), 0),
    whose sum the kernel takes as the fixed order-0 sum.  With w_i = +1 (x_i >= 0) else -1,
    K_j = sum_{i in R} w_i x_{i-j} and N = #{i in R: w_i = -1}, R = [lmax, hi) (hi = n: the
    whole bound; k_resid_sb's first test stops at hi = 8 * split * 512):
    LB_p = K_0 - floor(sum_j c_j K_j / 2^s) - 1 - N.  rec: the oracle's record in the L = 32
    layout (FLACMI_LPC_REC_WORDS(32): order p's coefficients at 2 + 32 + p(p-1)/2)."""
    x = np.asarray(x, dtype=np.int64)
    n = len(x)
    hi = n if hi is None else min(hi, n)
    w = np.where(x[lmax:hi] >= 0, 1, -1)
    K = [int(np.dot(w, x[lmax - j:hi - j])) for j in range(L + 1)]
    nneg = int((w < 0).sum())
    out = []
    for p in range(1, L + 1):
        if (int(rec[1]) >> (p - 1)) & 1:
            out.append(None)
            continue
        s = int(rec[2 + p - 1])
        base = 2 + 32 + p * (p - 1) // 2
        S = sum(int(rec[base + j]) * K[j + 1] for j in range(p))
        out.append(K[0] - (S >> s) - 1 - nneg)
    return out


def decides(x, rec, L, fixed_sums, lmax=32, split_end=None):
    """True when the bound proves every LPC order loses strictly to the best fixed sum: over
    R = [lmax, n), or (k_resid_sb, split_end given) first over [lmax, split_end)."""
    fmin = int(np.min(fixed_sums))

    def over(hi):
        for lb in order_bounds(x, rec, L, lmax, hi):
            if lb is None:
                if not int(fixed_sums[0]) > fmin:
                    return False
            elif not lb > fmin:
                return False
        return True
    return (split_end is not None and split_end < len(x) and over(split_end)) or over(None)
