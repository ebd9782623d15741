"""Child process of tests/test_gpu_lds_guard.py (run as a script, one process per kernel
variant: the variant switches FLACMI_NO_STREAM / FLACMI_NO_MFMA / FLACMI_NO_PRUNE /
FLACMI_POISON_LDS are read once per process).  Analyses fixed unit sets in several batch
arrangements and saves every result to an .npz for the parent to compare."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "oracle")]

import oracle  # noqa: E402  (the unit generator only)
from flac_amd.analysis import Analyzer, make_params  # noqa: E402


def unit_sets():
    """(name, rows, n, bits, params-list) for the kernel families: 16-bit 4608 (k_resid_stream,
    its retry list, the fast S16 / generic k_resid with 64 partitions), 24-bit 2048 at L = 32
    (PATH_W64 with int8-MFMA candidate sums) and a short 1024 block."""
    rng = np.random.default_rng(77)
    n = 4608
    t = np.arange(n)
    extra = []
    for u in range(6):
        w = rng.normal(0, 2000, n)
        ar = w.copy()
        ar[1:] += 0.9 * w[:-1]
        extra += [ar, rng.integers(-3000, 3000, n), 8000 * np.sin(2 * np.pi * (u + 1) * 37 / n * t)]
    extra += [np.zeros(n), np.full(n, 5.0)]
    s16 = np.concatenate([oracle.synth_batch(0, 30, n, 16, 31, dtype=np.int16),
                          np.clip(np.round(np.array(extra)), -32768, 32767).astype(np.int16)])
    s24 = oracle.synth_batch(0, 20, 2048, 24, 32, dtype=np.int32)
    s24[3, 100:] = 0
    s1k = oracle.synth_batch(0, 24, 1024, 16, 33, dtype=np.int16)
    # 16384 x 24-bit at L = 32 (config 3's shape): k_resid_sb decides the synthetic units, the
    # AR(1) and white-noise units go on to kVarList1 (planes and tiers), a top digit of 128
    # takes the int64 chains there, a silent block carries the LPC record's exception (the
    # round-4 fault was on the lazy plane build of this family)
    n3 = 16384
    s3 = oracle.synth_batch(0, 6, n3, 24, 34, dtype=np.int32)
    w3 = rng.normal(0, 2e5, (4, n3))
    w3[:2, 1:] += 0.9 * w3[:2, :-1]
    s3 = np.concatenate([s3, np.clip(np.round(w3), -2 ** 23, 2 ** 23 - 1).astype(np.int32)])
    s3[1, 5000] = 8355712
    s3[2, :] = 0
    return [
        ("s16", s16, n, 16, [(12, 5, 0, 5), (12, 9, 0, 5), (12, 5, 0, 6), (8, 5, 0, 5), (0, 5, 0, 5)]),
        ("s24", s24, 2048, 24, [(32, 15, 0, 6), (16, 12, 0, 5)]),
        ("s1k", s1k, 1024, 16, [(12, 5, 0, 4), (12, 5, 0, 6)]),
        ("s24k", s3, n3, 24, [(32, 15, 0, 8)]),
    ]


def arrangements(rows, seed):
    """(name, batch, index of each original unit in the batch): natural order, reversed,
    shuffled inside a larger batch of other units, and the first units one per call."""
    k = len(rows)
    rng = np.random.default_rng(seed)
    out = [("natural", [(rows, np.arange(k))]), ("reversed", [(rows[::-1].copy(), np.arange(k)[::-1].copy())])]
    filler = np.roll(rows, 3, axis=1)  # other units of the same shape and statistics
    big = np.concatenate([filler, rows, filler[: k // 2]])
    perm = rng.permutation(len(big))
    where = np.empty(k, dtype=np.int64)
    inv = np.argsort(perm)
    where[:] = inv[k + np.arange(k)]
    out.append(("embedded", [(big[perm].copy(), where)]))
    out.append(("single", [(rows[i:i + 1].copy(), np.array([0])) for i in range(min(4, k))]))
    return out


def main(path):
    az = Analyzer(0)
    res = {}
    for name, rows, n, bits, plist in unit_sets():
        for (L, q, rmin, rmax) in plist:
            mode = 1 if L == 0 else 0
            p = make_params(L, q, rmin, rmax, mode)
            for an, calls in arrangements(rows, 5):
                metas, resid, prm = [], [], []
                for batch, where in calls:
                    out = az.analyze(batch, p, n, sample_bits=bits)
                    for j, w in enumerate(where):
                        metas.append(out["meta"][w])
                        r = np.zeros(n + 8, dtype=np.uint64)
                        r[: out["residual"].shape[1]] = out["residual"][w]
                        resid.append(r)
                        prm.append(out["rice_params"][w])
                key = f"{name}|{L},{q},{rmin},{rmax}|{an}"
                res[key + "|meta"] = np.array(metas)
                res[key + "|residual"] = np.array(resid)
                res[key + "|params"] = np.array(prm)
    az.close()
    np.savez(path, **res)
    print("child ok", len(res))


if __name__ == "__main__":
    main(sys.argv[1])
