"""Device frame writer (csrc/k_frame.hip) against the frame-writer oracle
(oracle/frame_writer.py, pinned to the reference's streams by
tests/test_frame_writer_golden.py): every frame byte-identical, on the oracle's own
analysis of the same units, for the BASELINE config shapes and the header / writer edge
cases (explicit 8/16-bit block sizes, 1..6-byte coded numbers, frames larger than the
kernel's 16 KB LDS window, Rice5Bit, frame-number overflow, the q = 16 writer assert), and
frames that k_pack32 hands to the general k_pack."""
import numpy as np
import pytest

import frame_writer as FW
import oracle
from flac_amd import abi
from flac_amd.analysis import knob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def az():
    from flac_amd.analysis import Analyzer
    a = Analyzer(0)
    yield a
    a.close()


# (frames, channels, block, tail, bits, L, q, rmin, rmax, mode, sample_size, first_frame, seed)
CASES = {
    "c2": (48, 1, 4608, 0, 16, 12, 5, 0, 5, 0, 16, 0, 11),
    "c1_tail": (21, 1, 4608, 3240, 16, 8, 5, 0, 5, 0, 16, 75, 12),
    "c3_stereo": (4, 2, 16384, 0, 24, 32, 15, 0, 8, 0, 24, 1000, 13),
    "c3_tail": (3, 2, 16384, 1000, 24, 32, 15, 0, 8, 0, 24, 2047, 14),
    "c5_fixed": (48, 1, 4608, 0, 16, 0, 5, 0, 5, 1, 16, 65535, 15),
    "bs16_3ch": (12, 3, 1000, 77, 16, 12, 12, 0, 3, 0, 16, (1 << 21) - 5, 16),
    "bs8_coded6": (9, 2, 200, 100, 12, 8, 9, 0, 2, 0, 12, (1 << 31) - 12, 17),
    "q16_assert": (12, 1, 1152, 0, 16, 8, 16, 0, 4, 0, 16, 0, 18),
    "overflow": (6, 1, 576, 0, 16, 4, 5, 0, 3, 0, 16, (1 << 31) - 3, 19),
    "wide20": (6, 2, 4096, 0, 20, 12, 14, 0, 6, 0, 20, 9, 20),
    # frames > the 16 KB LDS window: with k_pack32 active (knob 2 / 7 below) handed to k_pack
    # by list
    "big3ch_list": (8, 3, 4608, 0, 20, 12, 12, 0, 5, 0, 20, 3, 21),
    # k_packw batches: a block that is not a multiple of 8 (the row's last chunk read value by
    # value), 5-value partitions (order 11 at 10240: every frame handed to k_pack by list), and
    # 16-bit stereo 16384-sample frames with a short last frame
    "wide_odd": (3, 2, 9001, 0, 16, 8, 12, 0, 4, 0, 16, 5, 22),
    "wide_fine": (3, 1, 10240, 0, 16, 0, 5, 11, 11, 1, 16, 7, 23),
    "wide16_tail": (3, 2, 16384, 5000, 16, 12, 12, 0, 8, 0, 16, 9, 24),
}


def _rows(frames, C, n, tail, bits, seed):
    dt = np.int16 if bits <= 16 else np.int32
    rows = oracle.synth_batch(seed * 1000, frames * C, n, bits, seed, dtype=dt)
    if tail:
        rows[-C:, tail:] = 0
    return rows, (C if tail else 0)


@pytest.mark.parametrize("name", sorted(CASES))
def test_frames_match_oracle_writer(az, name):
    frames, C, n, tail, bits, L, q, rmin, rmax, mode, ss, first, seed = CASES[name]
    rows, n_tail = _rows(frames, C, n, tail, bits, seed)
    params = oracle.make_params(L, q, rmin, rmax, mode)
    data, offsets, status = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C,
                                             sample_size=ss, first_frame=first)
    ora = oracle.analyze_batch(rows, params, n, tail, n_tail, sample_bits=bits, threads=8)
    want = FW.frames_from_analysis(rows, ora, C, n, tail, ss, q, first_frame=first)
    assert len(offsets) == frames + 1 and offsets[0] == 0
    for f, w in enumerate(want):
        st = int(status[f])
        if isinstance(w, Exception):
            assert st != 0, f"frame {f}: reference raises {type(w).__name__}, device wrote a frame"
            assert abi.STATUS_EXCEPTION[st & 0xFFFF] is type(w), f"frame {f}: status {st:#x} vs {w!r}"
            assert offsets[f + 1] == offsets[f]
            continue
        assert st == 0, f"frame {f}: device status {st:#x}, reference writes a frame"
        got = data[offsets[f]:offsets[f + 1]].tobytes()
        assert got == w, f"frame {f}: {len(got)} vs {len(w)} bytes, first diff at " \
                         f"{next((i for i in range(min(len(got), len(w))) if got[i] != w[i]), None)}"
    if name == "overflow":
        assert [int(s) >> 16 for s in status] == [0, 0, 0, 15, 15, 15]
    if name == "big3ch_list":
        assert (np.diff(offsets) + 8 > 4 * 4096).all()  # every frame takes the k_pack hand-off
    if name in ("c3_stereo", "c3_tail"):
        full = np.diff(offsets)[: frames - (1 if tail else 0)]
        assert (full > 4 * 4096).all()  # every full frame spans several 16 KB LDS windows


def test_device_pointer_path_matches_host_path(az):
    """flacmi_analyze_device + flacmi_frame_sizes_device + flacmi_pack_frames_device on
    device buffers give the bytes of flacmi_encode_host."""
    import torch
    from flac_amd.analysis import device_batch, frame_params, params_stride_for
    frames, C, n, L, q = 40, 2, 4608, 12, 5
    rows = oracle.synth_batch(777, frames * C, n, 16, 5, dtype=np.int16)
    params = oracle.make_params(L, q, 0, 5)
    data, offsets, status = az.encode_frames(rows, params, n, 0, 0, sample_bits=16, channels=C,
                                             sample_size=16, first_frame=3)
    dev = torch.device("cuda", 0)
    s = torch.as_tensor(rows, device=dev)
    pst = params_stride_for(5)
    meta = torch.empty((frames * C, abi.META_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    rp = torch.empty((frames * C, pst), dtype=torch.int32, device=dev)
    res = torch.empty((frames * C, n), dtype=torch.int32, device=dev)
    off = torch.empty(frames + 1, dtype=torch.int64, device=dev)
    st = torch.empty(frames, dtype=torch.int32, device=dev)
    out = torch.zeros(int(offsets[-1]) + 64, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    az.analyze_device(s.data_ptr(), 2, 16, n, frames * C, n, params, meta.data_ptr(), rp.data_ptr(), pst,
                      res.data_ptr(), n, 4, stream)
    b = device_batch(s.data_ptr(), 2, 16, n, frames * C, n)
    fp = frame_params(C, 16, q, 3)
    az.frame_sizes_device(b, fp, meta.data_ptr(), rp.data_ptr(), pst, off.data_ptr(), st.data_ptr(), stream)
    az.pack_frames_device(b, fp, meta.data_ptr(), rp.data_ptr(), pst, res.data_ptr(), 4, n, off.data_ptr(),
                          st.data_ptr(), out.data_ptr(), out.numel(), stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(off.cpu().numpy(), offsets)
    assert not st.cpu().numpy().any()
    assert out.cpu().numpy()[: int(offsets[-1])].tobytes() == data.tobytes()
    # too small an output buffer: nothing written, frame_status[0] says so
    small = torch.zeros(16, dtype=torch.uint8, device=dev)
    az.pack_frames_device(b, fp, meta.data_ptr(), rp.data_ptr(), pst, res.data_ptr(), 4, n, off.data_ptr(),
                          st.data_ptr(), small.data_ptr(), small.numel(), stream)
    torch.cuda.synchronize(dev)
    assert int(st[0].item()) == (17 << 16) | abi.STATUS_FRAME_TOO_LARGE
    assert not small.cpu().numpy().any()


@pytest.mark.parametrize("gen", [1, 2, 3, 7])
@pytest.mark.parametrize("name", ["c2", "c1_tail", "bs16_3ch", "c3_stereo", "c3_tail", "wide20", "wide_odd",
                                  "wide_fine", "wide16_tail", "big3ch_list", "c5_fixed", "bs8_coded6"])
def test_general_writer_alone_matches(az, name, gen):
    """Knob FLACMI_PACK_GENERIC=1 (every frame through the general k_pack) and =2 (k_packw
    off: k_pack32 for the frames it fits, k_pack for the rest) give the default path's bytes
    (k_packw for every 32-bit batch); the c3 frames exercise k_packw's ring against k_pack,
    and =3 (k_packw with tiles of 2048
    values, about 1400 ring words for these 24-bit frames) its redo of a segment that
    overruns the 1024-word ring; =7 keeps k_pack32 on its 16 KB window (the default takes
    the 12 KB window when a verbatim frame fits it with a quarter to spare)."""
    frames, C, n, tail, bits, L, q, rmin, rmax, mode, ss, first, seed = CASES[name]
    rows, n_tail = _rows(frames, C, n, tail, bits, seed)
    params = oracle.make_params(L, q, rmin, rmax, mode)
    want = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C, sample_size=ss,
                            first_frame=first)
    with knob("FLACMI_PACK_GENERIC", gen):
        got = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C, sample_size=ss,
                               first_frame=first)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])
    assert got[0].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("name,upb", [("c2", 5), ("c1_tail", 4), ("c3_stereo", 2), ("bs16_3ch", 3),
                                      ("q16_assert", 12), ("wide20", 4), ("big3ch_list", 6),
                                      ("wide_odd", 2), ("wide16_tail", 2)])
def test_encode_pipeline_equals_encode_frames(az, name, upb):
    """flacmi_encode_pipeline (sub-batches of upb frames, three in flight, the caller's
    buffers page-locked in place) gives the bytes, offsets and statuses of the one-shot
    flacmi_encode_host path, including the short last frame, the writer's own asserts
    and the 64-bit-residual redo; the rows are a strided view (row stride > block)."""
    frames, C, n, tail, bits, L, q, rmin, rmax, mode, ss, first, seed = CASES[name]
    rows, n_tail = _rows(frames, C, n, tail, bits, seed)
    params = oracle.make_params(L, q, rmin, rmax, mode)
    want = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C, sample_size=ss,
                            first_frame=first)
    wide = np.zeros((rows.shape[0], n + 40), dtype=rows.dtype)
    wide[:, :n] = rows
    view = wide[:, :n]  # row stride n + 40 samples
    data, offsets, status, timing = az.encode_pipeline(view, params, n, tail, n_tail, sample_bits=bits,
                                                       channels=C, sample_size=ss, first_frame=first,
                                                       units_per_batch=upb * C)
    assert np.array_equal(offsets, want[1]), name
    assert np.array_equal(status, want[2]), name
    assert data.tobytes() == want[0].tobytes(), name
    assert timing["sub_batches"] == (frames + upb - 1) // upb
    assert timing["bytes_out"] == int(offsets[-1])


def test_encode_pipeline_with_caller_pinned_buffers(az):
    """Rows and frame buffer page-locked once by the caller (flacmi_host_register): the
    pipeline uses them as they are (no per-call locking) and two calls through the same
    buffers give the one-shot path's bytes."""
    frames, C, n, tail, bits, L, q, rmin, rmax, mode, ss, first, seed = CASES["c2"]
    rows, n_tail = _rows(frames, C, n, tail, bits, seed)
    params = oracle.make_params(L, q, rmin, rmax, mode)
    want = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C, sample_size=ss,
                            first_frame=first)
    rows = np.ascontiguousarray(rows)
    out = np.zeros(len(want[0]) + 4096, dtype=np.uint8)
    az.host_register(rows)
    az.host_register(out)
    try:
        for _ in range(2):
            data, offsets, status, t = az.encode_pipeline(rows, params, n, tail, n_tail, sample_bits=bits,
                                                          channels=C, sample_size=ss, first_frame=first,
                                                          units_per_batch=5 * C, out=out)
            assert np.array_equal(offsets, want[1]) and np.array_equal(status, want[2])
            assert data.tobytes() == want[0].tobytes()
            assert t["register_ms"] < 50.0
    finally:
        az.host_unregister(out)
        az.host_unregister(rows)
