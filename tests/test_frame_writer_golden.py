"""Pin the frame-writer oracle (oracle/frame_writer.py) to the reference: whole streams
rebuilt from the C oracle's analysis + the writer restatement must hash to the
reference encode() output recorded in tests/golden/streams.json (made by
tests/golden/make_golden.py from the reference itself)."""
import hashlib
import math

import numpy as np
import pytest

import frame_writer as FW
import golden_util as G
import oracle


def _stream(pcm_channels, block, sample_rate, sample_size, L, q, rmin, rmax):
    chans = [np.asarray(c, dtype=np.int64) for c in pcm_channels]
    C, total = len(chans), len(chans[0])
    nb = (total + block - 1) // block
    tail = total - (nb - 1) * block
    dt = np.int16 if sample_size <= 16 else np.int32
    rows = np.zeros((nb * C, block), dtype=dt)
    for b in range(nb):
        for c in range(C):
            seg = chans[c][b * block:(b + 1) * block]
            rows[b * C + c, :len(seg)] = seg
    n_tail = C if tail != block else 0
    out = oracle.analyze_batch(rows, oracle.make_params(L, q, rmin, rmax), block, tail if n_tail else 0, n_tail,
                               sample_bits=sample_size, threads=8)
    frames = FW.frames_from_analysis(rows, out, C, block, tail if n_tail else 0, sample_size, q)
    assert all(isinstance(f, bytes) for f in frames)
    data = FW.stream_header(sample_rate, sample_size, C, total, block) + b"".join(frames)
    return len(data), hashlib.sha256(data).hexdigest()


def _sine(n):
    return [round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n)]


@pytest.mark.parametrize("name", ["c1_correct", "c1_quirk"])
def test_c1_streams(name):
    S = G.load("streams.json")
    pcm = _sine(441000)
    if name == "c1_quirk":  # flac/__main__.py's reader hands encode() the low byte as int8
        pcm = [((v & 0xFF) ^ 0x80) - 0x80 for v in pcm]
    assert G.samples_sha(pcm) == S[name]["samples_sha256"]
    assert _stream([pcm], 4608, 44100, 16, 8, 5, 0, 5) == (S[name]["len"], S[name]["sha256"])


def test_c3_stereo_stream():
    e = G.load("streams.json")["c3_stereo"]
    n = e["frames"]
    chans = [oracle.synth_unit(c["unit"], n, e["sample_size"], c["seed"]) for c in e["channels"]]
    got = _stream(chans, e["block_size"], e["sample_rate"], e["sample_size"], e["max_lpc_order"],
                  e["qlp_precision"], e["rice"][0], e["rice"][1])
    assert got == (e["len"], e["sha256"])


def test_writer_pieces():
    # CRC-8/CRC-16 (FLAC polynomials, init 0) of "123456789"
    assert FW.crc8(b"123456789") == 0xF4 and FW.crc16(b"123456789") == 0xFEE8
    assert FW.coded_number(0b10101010_101) == bytes([0b11010101, 0b10010101])
    with pytest.raises(ValueError):
        FW.coded_number(1 << 31)
    h = FW.frame_header(95, 3240)
    assert h[2] >> 4 == 0b0111 and int.from_bytes(h[5:7], "big") == 3239
    assert FW.frame_header(0, 4608)[:4] == bytes([0xFF, 0xF8, 0x50, 0x10])
    packed, nb = FW.rice_packed([5, 0, 9], [1, 0, 2])
    # 5,p=1: q=2 -> 00 1 1 ; 0,p=0: 1 ; 9,p=2: q=2 -> 00 1 01
    assert nb == 4 + 1 + 5 and packed == bytes([0b00111001, 0b01000000])
