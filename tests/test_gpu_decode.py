"""Device decoder verifier (csrc/k_decode.hip, flacmi_decode_frames_device).

1. Golden: every frame of tests/golden/decode.json (assembled by make_decode_golden.py and
   read back by the reference's own get_frame + decode_frame) decodes to the reference's
   samples, or fails with the reference's exception class at the expected statement.
2. Round trip (BASELINE config 5 and the other config shapes): frames written by the
   device encoder decode on the device to exactly the source units, with CRC-8/16, frame
   numbers, frame ends and block sizes verified, and a corrupted byte is caught.
Every test runs twice: with k_decode_fx taking the frames it accepts (the default) and with
the FLACMI_DECODE_GENERIC knob sending every frame through the general k_decode.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from flac_amd import abi
from flac_amd.analysis import knob

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "decode.json")


@pytest.fixture(scope="module", params=["fx", "generic"])
def az(request):
    from flac_amd.analysis import Analyzer
    a = Analyzer(0)
    with knob("FLACMI_DECODE_GENERIC", int(request.param == "generic")):
        yield a
    a.close()


def _golden():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _golden(), ids=lambda c: c["name"])
def test_decoder_matches_reference_decoder(az, case):
    data = np.frombuffer(bytes.fromhex(case["hex"]), dtype=np.uint8)
    offsets = np.array([0, len(data)], dtype=np.int64)
    out, st, mm = az.decode_frames(data, offsets, case["channels"], case["sample_size"], first_frame=-1,
                                   block_len=32768, out_stride=32768)
    st = int(st[0])
    if case["exception"] is not None:
        assert st != 0, f"reference raises {case['exception']}, device decoded the frame"
        assert abi.STATUS_EXCEPTION[st & 0xFFFF].__name__ == case["exception"], f"status {st:#x}"
        if case["site"]:
            assert st >> 16 == abi.DSITE[case["site"]], f"site {st >> 16} != {case['site']}"
        return
    if case["verify"]:
        assert st == (abi.DSITE[case["verify"]] << 16) | abi.STATUS_VERIFY, f"status {st:#x}"
    else:
        assert st == 0, f"status {st:#x} (site {st >> 16})"
    bs = case["block_size"]
    dec = out[: case["channels"], :bs].astype(np.int64)
    assert [list(r[:8]) for r in dec] == case["decoded_head"]
    assert hashlib.sha256(dec.astype("<i8").tobytes()).hexdigest() == case["decoded_sha256"]


# (frames, channels, block, tail, bits, L, q, rmin, rmax, mode, sample_size, first_frame, seed)
ROUND_TRIP = {
    "c2": (64, 1, 4608, 0, 16, 12, 5, 0, 5, 0, 16, 0, 31),
    "c1_tail": (21, 1, 4608, 3240, 16, 8, 5, 0, 5, 0, 16, 75, 32),
    "c3_stereo": (4, 2, 16384, 0, 24, 32, 15, 0, 8, 0, 24, 1000, 33),
    "c3_tail": (3, 2, 16384, 1000, 24, 32, 15, 0, 8, 0, 24, 2047, 34),
    "c5_fixed": (200, 1, 4608, 0, 16, 0, 5, 0, 5, 1, 16, 65535, 35),
    "bs16_3ch": (12, 3, 1000, 77, 16, 12, 12, 0, 3, 0, 16, (1 << 21) - 5, 36),
    "wide20": (6, 2, 4096, 0, 20, 12, 14, 0, 6, 0, 20, 9, 37),
    "lpc_heavy_q15": (40, 1, 4096, 0, 16, 32, 15, 0, 8, 0, 16, 5, 38),
}


def _encode(az, name):
    frames, C, n, tail, bits, L, q, rmin, rmax, mode, ss, first, seed = ROUND_TRIP[name]
    dt = np.int16 if bits <= 16 else np.int32
    rows = oracle.synth_batch(seed * 1000, frames * C, n, bits, seed, dtype=dt)
    n_tail = C if tail else 0
    if tail:
        rows[-C:, tail:] = 0
    params = oracle.make_params(L, q, rmin, rmax, mode)
    data, offsets, status = az.encode_frames(rows, params, n, tail, n_tail, sample_bits=bits, channels=C,
                                             sample_size=ss, first_frame=first)
    assert not status.any(), "round-trip shapes are chosen so the reference writes every frame"
    return rows, data, offsets, (C, n, tail, n_tail, ss, first)


@pytest.mark.parametrize("name", sorted(ROUND_TRIP))
def test_round_trip_bit_exact(az, name):
    rows, data, offsets, (C, n, tail, n_tail, ss, first) = _encode(az, name)
    out, st, mm = az.decode_frames(data, offsets, C, ss, first_frame=first, expect=rows, block_len=n,
                                   tail_len=tail, n_tail_units=n_tail)
    assert not st.any(), f"frames with status: {[(i, hex(int(s))) for i, s in enumerate(st) if s][:5]}"
    assert not mm.any()
    for u in range(rows.shape[0]):
        ln = tail if (n_tail and u >= rows.shape[0] - n_tail) else n
        assert np.array_equal(out[u, :ln], rows[u, :ln].astype(np.int32)), f"unit {u}"
    if name == "c5_fixed":  # every subframe of the fixed-only stream is FIXED (type byte 0b0001xxx0)
        from flac_amd.coded_number import required_bytes
        for i, o in enumerate(offsets[:-1]):
            assert data[int(o) + 4 + required_bytes(first + i) + 1] >> 4 == 1, f"frame {i}"


def test_corruption_is_caught(az):
    rows, data, offsets, (C, n, tail, n_tail, ss, first) = _encode(az, "c2")
    bad = data.copy()
    f = 7
    mid = (int(offsets[f]) + int(offsets[f + 1])) // 2
    bad[mid] ^= 0x10
    _, st, mm = az.decode_frames(bad, offsets, C, ss, first_frame=first, expect=rows, block_len=n)
    assert [i for i, s in enumerate(st) if s] == [f]
    # a flipped residual bit either breaks the parse or changes samples; never silent
    assert mm[f] > 0 or (int(st[f]) >> 16) in (abi.DSITE["frame_end"], abi.DSITE["eof"], abi.DSITE["padding"],
                                                abi.DSITE["crc16"], abi.DSITE["partitions"])
    # frame numbers are checked against first_frame
    _, st2, _ = az.decode_frames(data, offsets, C, ss, first_frame=first + 1, block_len=n)
    assert all((int(s) >> 16) == abi.DSITE["frame_number"] for s in st2)
    # without the CRC / number checks the clean stream is accepted as the reference would
    _, st3, _ = az.decode_frames(data, offsets, C, ss, first_frame=-1, block_len=n, check_crc=False)
    assert not st3.any()


def test_crc16_fused_in_the_bit_reader(az):
    """k_decode folds each frame's CRC-16 as whole dwords leave its bit window (head and tail
    bytes apart).  Flipping a bit of the stored CRC-16 of frames at every byte alignment
    flags exactly those frames (crc16); the clean stream passes."""
    rows, data, offsets, (C, n, tail, n_tail, ss, first) = _encode(az, "c2")
    nf = len(offsets) - 1
    picks = []
    for al in range(4):  # up to four frames starting at each byte alignment
        picks += [f for f in range(nf) if int(offsets[f]) % 4 == al][:4]
    assert {int(offsets[f]) % 4 for f in picks} == {0, 1, 2, 3}
    bad = data.copy()
    for k, f in enumerate(picks):
        bad[int(offsets[f + 1]) - 1 - (k & 1)] ^= 0x01 << (k % 8)
    _, st, mm = az.decode_frames(bad, offsets, C, ss, first_frame=first, expect=rows, block_len=n)
    assert sorted(i for i, s in enumerate(st) if s) == sorted(picks)
    assert all((int(st[f]) >> 16) == abi.DSITE["crc16"] for f in picks)
    assert not mm.any()


def test_fast_and_general_decoders_agree_on_damaged_streams(az):
    """k_decode_fx hands every frame it cannot vouch for to k_decode: on a stream with LPC
    frames and bytes damaged at many places, the default split and the all-general run give
    the same status and mismatch count for every frame, and the same samples where status is 0."""
    rng = np.random.default_rng(5)
    for name in ("lpc_heavy_q15", "c2", "wide20"):
        rows, data, offsets, (C, n, tail, n_tail, ss, first) = _encode(az, name)
        bad = data.copy()
        nf = len(offsets) - 1
        hit = rng.choice(nf, size=max(3, nf // 4), replace=False)
        for f in hit:
            o0, o1 = int(offsets[f]), int(offsets[f + 1])
            pos = int(rng.integers(o0, o1))
            bad[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        res = {}
        for gen in (0, 1):
            with knob("FLACMI_DECODE_GENERIC", gen):
                res[gen] = az.decode_frames(bad, offsets, C, ss, first_frame=first, expect=rows, block_len=n,
                                            tail_len=tail, n_tail_units=n_tail)
        (o0, s0, m0), (o1, s1, m1) = res[0], res[1]
        assert np.array_equal(s0, s1), name
        assert np.array_equal(m0, m1), name
        assert s0.any(), name
        for f in range(nf):
            if s0[f] == 0:
                assert np.array_equal(o0[f * C:(f + 1) * C], o1[f * C:(f + 1) * C]), (name, f)
