"""numpy restatement of the k_stats kernel (flac-py_amd/csrc/k_misc.hip): the 128-word
stream-statistics vector that bench.py all-reduces over ranks.  Test infrastructure."""
import numpy as np

M64 = (1 << 64) - 1


def stream_stats(meta, block_len, tail_len=0, n_tail_units=0):
    h = [0] * 128
    nu = len(meta)
    for u in range(nu):
        m = meta[u]
        n = tail_len if u >= nu - n_tail_units else block_len
        h[0] += 1
        h[1] += n
        st = int(m["status"])
        h[64 + (15 if st >= 16 else st & 15)] += 1
        if st != 0:
            continue
        h[2] += int(m["rice_bits"])
        order = int(m["order"])
        if int(m["kind"]) == 0:
            h[3] += 1
            h[5 + (order & 7) % 5] += 1
        else:
            h[4] += 1
            h[9 + (order if 1 <= order <= 32 else 32)] += 1
        h[48 + (int(m["part_order"]) & 15)] += 1
        h[81] += int(m["lpc_order"]) == -1
        hsh = ((int(m["rice_bits"]) * 0x9E3779B97F4A7C15) & M64) ^ ((int(m["fixed_sum"]) << 1) & M64) ^ \
            (((int(m["kind"]) * 64 + order) * 0xD1B54A32D192ED03) & M64)
        h[80] = (h[80] + hsh) & M64
    out = np.array([v if v < (1 << 63) else v - (1 << 64) for v in h], dtype=np.int64)
    return out
