"""Debug helper (GPU box): analyse synthetic / sine units on the device and print the
first fields that differ from the oracle."""
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import oracle  # noqa: E402
from flac_amd import abi  # noqa: E402
from flac_amd.analysis import Analyzer, make_params  # noqa: E402


def cmp(name, a, n, L, q, rmin, rmax, mode=0, bits=16):
    az = Analyzer(0)
    g = az.analyze(a, make_params(L, q, rmin, rmax, mode), n, sample_bits=bits, debug=True)
    o = oracle.analyze_batch(a, oracle.make_params(L, q, rmin, rmax, mode), n, sample_bits=bits, threads=8)
    gm, om = g["meta"], o["meta"]
    bad = 0
    for u in range(len(a)):
        diffs = [f for f in abi.META_DTYPE.names if not np.array_equal(gm[f][u], om[f][u])]
        off, ln = int(om["res_offset"][u]), int(om["res_len"][u])
        if not np.array_equal(g["residual"][u][off:off + ln].astype(np.uint64), o["residual"][u][off:off + ln]):
            diffs.append("residual")
        k = int(om["n_parts"][u])
        if not np.array_equal(g["rice_params"][u][:k], o["rice_params"][u][:k]):
            diffs.append("rice_params")
        if not np.array_equal(g["fixed_sums"][u], o["fixed_sums"][u]):
            diffs.append("fixed_sums")
        if not np.array_equal(g["lpc_sums"][u], o["lpc_sums"][u]):
            diffs.append("lpc_sums")
        if diffs:
            bad += 1
            if bad <= 4:
                print(f"[{name}] unit {u}: {diffs}")
                for f in diffs:
                    if f in abi.META_DTYPE.names:
                        print("   ", f, "gpu", gm[f][u], "ora", om[f][u])
                    elif f in ("fixed_sums", "lpc_sums"):
                        print("   ", f, "gpu", g[f][u][:13], "ora", o[f][u][:13])
                    elif f == "residual":
                        d = np.nonzero(g["residual"][u][off:off + ln].astype(np.uint64) != o["residual"][u][off:off + ln])[0]
                        print("    residual first diffs at", d[:8], g["residual"][u][off + d[:4]], o["residual"][u][off + d[:4]])
    print(f"[{name}] {bad} of {len(a)} units differ")
    az.close()


if __name__ == "__main__":
    n = 4608
    sine = np.array([round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n * 8)],
                    dtype=np.int16).reshape(8, n)
    cmp("sine L8", sine, n, 8, 5, 0, 5)
    a = oracle.synth_batch(0, 256, n, 16, 2024, dtype=np.int16)
    cmp("c2", a, n, 12, 5, 0, 5)
    cmp("c5", a, n, 0, 5, 0, 5, mode=1)
    cmp("c2 L8", a, n, 8, 5, 0, 5)
    cmp("c2 L4", a, n, 4, 5, 0, 5)
