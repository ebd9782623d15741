"""Multi-GPU contract on one GPU: the config-2 job analysed as
G = 1/2/4/8 logical shards, each shard generated and analysed on its own exactly as one
bench.py rank does it (bench.shard_plan -> synth_device(first_unit) -> analyze_device ->
stream_stats), gives the unsharded run's meta, residual rows and Rice parameters, and the
per-shard 128-word stream statistics sum to the unsharded vector (what the RCCL
all-reduce adds up).  Units are independent and the frame number is the block index
(reference flac/encoder.py:87-97), so sharding must not change a single bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U, N, BITS, SEED = 12_000, 4608, 16, 2024


def _run(az, first, units, params, dev):
    import torch
    from flac_amd import abi
    from flac_amd.analysis import params_stride_for
    sstride = ((N * 2 + 15) // 16) * 16 // 2
    rstride = ((N * 4 + 15) // 16) * 16 // 4
    pstride = params_stride_for(params.rice_max)
    s = torch.empty((units, sstride), dtype=torch.int16, device=dev)
    meta = torch.empty((units, abi.META_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    rp = torch.zeros((units, pstride), dtype=torch.int32, device=dev)
    res = torch.zeros((units, rstride), dtype=torch.int32, device=dev)
    st = torch.zeros(abi.STATS_WORDS, dtype=torch.int64, device=dev)
    az.synth_device(s.data_ptr(), 2, BITS, sstride, first, units, N, SEED)
    az.analyze_device(s.data_ptr(), 2, BITS, sstride, units, N, params, meta.data_ptr(), rp.data_ptr(), pstride,
                      res.data_ptr(), rstride, 4)
    az.stream_stats(meta.data_ptr(), units, N, st.data_ptr())
    torch.cuda.synchronize(dev)
    return meta.cpu().numpy(), rp.cpu().numpy(), res, st.cpu().numpy()


def test_logical_shards_equal_unsharded():
    import torch

    import bench
    from flac_amd.analysis import Analyzer, make_params

    dev = torch.device("cuda", 0)
    az = Analyzer(0)
    cfg = bench.CONFIGS["c2"]
    params = make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])
    m0, p0, r0, s0 = _run(az, 0, U, params, dev)
    for G in (1, 2, 4, 8):
        per = U // G
        stats = np.zeros_like(s0)
        for g in range(G):
            first, chunks, total = bench.shard_plan(cfg, g, G, per)
            assert not chunks and total == U and first == g * per
            m, p, r, s = _run(az, first, per, params, dev)
            sl = slice(first, first + per)
            assert np.array_equal(m, m0[sl]), f"G={G} shard {g}: meta differs"
            assert np.array_equal(p, p0[sl]), f"G={G} shard {g}: Rice parameters differ"
            assert torch.equal(r, r0[sl]), f"G={G} shard {g}: residual rows differ"
            stats += s
        assert stats.tolist() == s0.tolist(), f"G={G}: summed shard statistics differ from the unsharded run"
    assert s0[0] == U and s0[1] == U * N
    az.close()
