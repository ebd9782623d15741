"""Per-unit phase latencies of k_resid_stream from the diagnostic build
(libflacmi_stamps.so, -DFLACMI_STREAM_STAMPS=1: wave 0 stamps s_memtime at each phase
boundary into lpc_sums[.., 24:32] and s_memrealtime into fixed_sums[.., 3:5]).
Usage: FLACMI_LIB=$PWD/flac-py_amd/libflacmi_stamps.so python tools/stamps.py [units] [config]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch

    import bench
    from flac_amd.analysis import Analyzer, make_params
    units = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    cfg = bench.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c2"]
    n = 4608
    az = Analyzer(0)
    sstride = ((n * 2 + 15) // 16) * 16 // 2
    s = torch.empty((units, sstride), dtype=torch.int16, device="cuda:0")
    az.synth_device(s.data_ptr(), 2, 16, sstride, 0, units, n, 2024)
    torch.cuda.synchronize()
    host = s.cpu().numpy()
    params = make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])
    for rep in range(2):
        out = az.analyze(host, params, n, debug=True)
    st = out["lpc_sums"][:, 24:32].astype(np.int64)
    rt = out["fixed_sums"][:, 3:5].astype(np.int64)
    ok = (st[:, 7] > 0) & (st[:, 0] > 0)
    st, rt = st[ok], rt[ok]
    d = np.diff(st, axis=1)
    names = ["staging loads", "B1 wait", "status+MFMA+B2", "choice", "residual+B3", "Rice+B4", "final (wave 0)"]
    life = st[:, 7] - st[:, 0]
    clk = life.sum() / ((rt[:, 1] - rt[:, 0]).sum() / 100e6) / 1e9
    print(f"units {ok.sum()} of {units}; shader clock {clk:.2f} GHz; lifetime median {np.median(life):.0f} cyc,"
          f" mean {life.mean():.0f}")
    for i, nm in enumerate(names):
        print(f"  {nm:18s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  p90 {np.percentile(d[:, i], 90):8.0f}")
    span = (rt[:, 1].max() - rt[:, 0].min()) / 100e6
    inflight = ((rt[:, 1] - rt[:, 0]) / 100e6).sum() / span
    print(f"kernel span {span * 1e3:.2f} ms, mean units in flight {inflight:.0f} ({inflight / 256:.1f} per CU)")


if __name__ == "__main__":
    main()
