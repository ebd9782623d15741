"""BASELINE config 4's own code path on one GPU: the job of N blocks generated on the device
in chunks, chunk ci going to rank ci % W (bench.shard_plan round-robin), each rank running
bench.run_chunks (synth_device -> analyze_device -> stream_stats per chunk) exactly as a
bench.py rank does.  For W = 1/2/4/8 logical ranks the per-rank statistics must sum to the
W = 1 vector (what the RCCL all-reduce adds up), the chunk assignment must cover the job
once, and sampled units of every chunk (first, last, random) must equal the CPU oracle on
the same generated blocks.  Units are independent and the frame number is the block index
(reference flac/encoder.py:87-99), so the split must not change a bit."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

TOTAL, CHUNK = 205_000, 20_000  # 11 chunks, the last one short (5,000 blocks)


def test_c4_round_robin_chunks_equal_single_rank():
    import torch

    import bench
    from flac_amd import abi
    from flac_amd.analysis import Analyzer, make_params, params_stride_for

    dev = torch.device("cuda", 0)
    az = Analyzer(0)
    cfg = bench.CONFIGS["c4"]
    n, bits = cfg["n"], cfg["bits"]
    params = make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])
    sstride = ((n * 2 + 15) // 16) * 16 // 2
    rstride = ((n * 4 + 15) // 16) * 16 // 4
    pstride = params_stride_for(cfg["rmax"])
    bufs = dict(samples=torch.empty((CHUNK, sstride), dtype=torch.int16, device=dev),
                meta=torch.empty((CHUNK, abi.META_DTYPE.itemsize), dtype=torch.uint8, device=dev),
                rparams=torch.empty((CHUNK, pstride), dtype=torch.int32, device=dev),
                residual=torch.empty((CHUNK, rstride), dtype=torch.int32, device=dev),
                stats=torch.zeros(abi.STATS_WORDS, dtype=torch.int64, device=dev),
                stats_acc=torch.zeros(abi.STATS_WORDS, dtype=torch.int64, device=dev))
    stream = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(4)
    checked = []

    def sample_chunk(ci, cu):
        """first, last and two random units of the chunk against the oracle"""
        torch.cuda.synchronize(dev)
        pick = sorted({0, cu - 1, *rng.integers(0, cu, 2).tolist()})
        rows = bufs.get("cur_samples", bufs["samples"])[pick].cpu().numpy()[:, :n]
        want = oracle.synth_batch(ci * CHUNK + pick[0], 1, n, bits, 2024)[0]
        assert np.array_equal(rows[0], want), f"chunk {ci}: generated block differs from the oracle's"
        ora = oracle.analyze_batch(np.ascontiguousarray(rows), oracle.make_params(cfg["L"], cfg["q"], cfg["rmin"],
                                   cfg["rmax"], cfg["mode"]), n, sample_bits=bits, threads=8)
        meta = bufs["meta"][pick].cpu().numpy().view(abi.META_DTYPE).reshape(len(pick))
        res = bufs["residual"][pick].cpu().numpy().view(np.uint32)
        rp = bufs["rparams"][pick].cpu().numpy()
        for j in range(len(pick)):
            bad = oracle.meta_mismatches(meta[j], ora["meta"][j])
            assert not bad, (ci, pick[j], bad)
            off, ln = int(meta[j]["res_offset"]), int(meta[j]["res_len"])
            assert np.array_equal(res[j][off:off + ln].astype(np.uint64), ora["residual"][j][off:off + ln])
            k = int(meta[j]["n_parts"])
            assert np.array_equal(rp[j][:k], ora["rice_params"][j][:k])
        checked.append(ci)

    whole = None
    for W in (1, 2, 4, 8):
        total = np.zeros(abi.STATS_WORDS, dtype=np.int64)
        seen = []
        for r in range(W):
            first, chunks, tot = bench.shard_plan(cfg, r, W, CHUNK, TOTAL)
            assert first == 0 and tot == TOTAL and chunks == list(range(r, 11, W))
            seen += chunks
            st = bench.run_chunks(az, cfg, params, bufs, chunks, CHUNK, TOTAL, 2024, stream,
                                  on_chunk=sample_chunk if W == 1 else None)
            torch.cuda.synchronize(dev)
            total += st.cpu().numpy()
        assert sorted(seen) == list(range(11)), f"W={W}: chunks not covered exactly once"
        if whole is None:
            whole = total
            assert whole[0] == TOTAL and whole[1] == TOTAL * n
            assert whole[64] == TOTAL, "config-4 units raise no exception"
        else:
            assert total.tolist() == whole.tolist(), f"W={W}: summed rank statistics differ from one rank"
    assert checked == list(range(11))
    # bench.py's double-buffered chunk loop (the next chunk generated on a side stream while
    # this one is analysed): same statistics at W = 1 and 2, and every chunk's sampled units
    # equal to the oracle
    bufs["samples_b"] = torch.empty_like(bufs["samples"])
    bufs["synth_stream"] = torch.cuda.Stream(dev)
    checked.clear()
    for W in (1, 2):
        total = np.zeros(abi.STATS_WORDS, dtype=np.int64)
        for r in range(W):
            _, chunks, _ = bench.shard_plan(cfg, r, W, CHUNK, TOTAL)
            st = bench.run_chunks(az, cfg, params, bufs, chunks, CHUNK, TOTAL, 2024, stream,
                                  on_chunk=sample_chunk if W == 1 else None)
            torch.cuda.synchronize(dev)
            total += st.cpu().numpy()
        assert total.tolist() == whole.tolist(), f"double-buffered W={W}: statistics differ"
    assert checked == list(range(11))
    az.close()
