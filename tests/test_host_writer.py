"""Host-side bitstream pieces (binary.Put/Get, CRC, coded numbers, Rice packing, header
writers) against byte patterns.  The Put/Get/coded-number vectors restate the cases of
the reference's own tests (test/test_binary.py, test/test_coded_number.py) as data."""
import io

import numpy as np
import pytest

from flac_amd import coded_number
from flac_amd.binary import Get, Put, extract, mask
from flac_amd.common import (CRC8_POLYNOMIAL, CRC16_POLYNOMIAL, BlockingStrategy, Channels,
                             FrameHeader, MetadataBlockHeader, MetadataBlockType, Streaminfo)
from flac_amd.crc import crc8, crc16
from flac_amd.utils import argparse_range, batch, group, zigzag_decode, zigzag_encode


def test_mask_extract():
    assert [mask(i) for i in range(4)] == [0, 1, 3, 7]
    assert extract(0b1, 1, 0, 1) == 1
    assert extract(0b10101010, 8, 0, 8) == 0b10101010
    assert extract(0b10101010, 8, 2, 5) == 0b101


@pytest.mark.parametrize("data,reads", [
    ((0b11010010_00100001_00000100_00001000_00001000_00000111).to_bytes(6, "big"),
     [(1, 0b1), (2, 0b10), (3, 0b100), (4, 0b1000), (5, 0b10000), (6, 0b100000), (7, 0b1000000),
      (8, 0b10000000), (9, 0b100000000), (3, 0b111)]),
    ((0b10000000_00000001).to_bytes(2, "big"), [(16, 0b10000000_00000001)]),
    ((0b00010000_00000000_00000000_00001111).to_bytes(4, "big"),
     [(3, 0), (25, 0b10000_00000000_00000000_0000), (4, 0b1111)]),
    (b"fLaC", [(32, int.from_bytes(b"fLaC", "big"))]),
])
def test_get(data, reads):
    g = Get(io.BytesIO(data))
    for n, want in reads:
        assert g.uint(n) == want


@pytest.mark.parametrize("writes,expect", [
    ([(0b10101010, 8), (0b01010101, 8)], bytes([0b10101010, 0b01010101])),
    ([(0b1, 1), (0b01, 2), (0b010, 3), (0b10, 2)], bytes([0b10101010])),
    ([(0b10000, 5), (0b11111111, 8), (0b001, 3)], bytes([0b10000111, 0b11111001])),
    ([(0b1000, 4), (0xFFFF, 16), (0b0001, 4)], bytes([0b10001111, 0xFF, 0b11110001])),
    ([(0, 16), (0, 16), (0, 24), (0, 24), (0, 20), (0b111, 3), (0b11111, 5), (0b1, 4)],
     bytes(12) + bytes([0b00001111, 0b11110001])),
    ([(-1, 5), (-6, 3)], bytes([0b11111010])),  # two's complement fields (warm-up, coefficients)
])
def test_put(writes, expect):
    p = Put()
    for x, n in writes:
        p.uint(x, n)
    assert p.is_aligned and p.buffer == expect


@pytest.mark.parametrize("decoded,encoded,size", [
    (0b00000000, 0b00000000, 1), (0b00011111, 0b00011111, 1), (0b01111111, 0b01111111, 1),
    (0b10000000, 0b11000010_10000000, 2), (0b10101010_1, 0b11000101_10010101, 2),
    (0b10101010_101, 0b11010101_10010101, 2)])
def test_coded_number(decoded, encoded, size):
    assert int.from_bytes(coded_number.encode(decoded), "big") == encoded
    assert coded_number.decode(encoded.to_bytes(size, "big")) == decoded


def test_coded_number_round_trip_all_sizes():
    for x in [0, 1, 127, 128, 2047, 2048, 65535, 65536, (1 << 21) - 1, 1 << 21, (1 << 26) - 1,
              1 << 26, (1 << 31) - 1]:
        assert coded_number.decode(coded_number.encode(x)) == x
    with pytest.raises(ValueError):
        coded_number.encode(1 << 31)


def test_crc_known_values():
    # CRC-8/CRC-16 (FLAC polynomials, init 0) of "123456789"
    assert crc8(b"123456789", CRC8_POLYNOMIAL) == 0xF4
    assert crc16(b"123456789", CRC16_POLYNOMIAL) == 0xFEE8


def test_rice_packed_matches_bit_serial():
    import frame_writer as FW  # the frame-writer oracle (test infrastructure)
    rng = np.random.default_rng(0)
    x = rng.integers(0, 3000, size=500).astype(np.uint64)
    p = rng.integers(0, 9, size=500)
    packed, nbits = FW.rice_packed(x, p)
    ref = Put()
    for v, k in zip(x.tolist(), p.tolist()):
        ref.uint(0, v >> k)
        ref.uint(1, 1)
        for i in reversed(range(k)):
            ref.uint((v >> i) & 1, 1)
    pad = (8 - nbits % 8) % 8
    ref.uint(0, pad)
    assert ref.buffer == packed


def test_utils():
    assert argparse_range("5") == range(0, 6) and argparse_range("2,5") == range(2, 6)
    with pytest.raises(AssertionError):
        argparse_range("0,0")
    assert [b for b in batch(iter("ABCDEFG"), 3)] == [["A", "B", "C"], ["D", "E", "F"], ["G"]]
    assert group([1, 2, 3, 4, 5, 6], 2) == [[1, 2], [3, 4], [5, 6]]
    for v in [0, 1, -1, 2, -2, 12345, -12345, (1 << 40), -(1 << 40)]:
        assert zigzag_decode(zigzag_encode(v)) == v
    assert [zigzag_encode(v) for v in (0, -1, 1, -2, 2)] == [0, 1, 2, 3, 4]


def test_stream_headers():
    from flac_amd.encoder import (put_frame_header, put_metadata_block_header,
                                  put_metadata_block_streaminfo)
    h = put_metadata_block_header(MetadataBlockHeader(True, MetadataBlockType.Streaminfo, 34)).buffer
    assert h == bytes([0x80, 0, 0, 34])
    si = put_metadata_block_streaminfo(Streaminfo(4608, 4608, 0, 0, 44100, 1, 16, 441000, bytes(16))).buffer
    assert len(si) == 34 and si[:4] == bytes([0x12, 0x00, 0x12, 0x00])
    fh = put_frame_header(FrameHeader(BlockingStrategy.Fixed, 4608, None, Channels.L_R, None, 0)).buffer
    assert fh[:4] == bytes([0xFF, 0xF8, 0x50, 0x10]) and len(fh) == 6
    fh = put_frame_header(FrameHeader(BlockingStrategy.Fixed, 3240, None, Channels.L_R, None, 95)).buffer
    assert fh[2] >> 4 == 0b0111 and int.from_bytes(fh[5:7], "big") == 3239
