"""CPU restatement of flac-py's frame writer — the checker of the device frame writer
(flac-py_amd/csrc/k_frame.hip).

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's checker leg.  The product
never imports this module.

Restates, on the per-unit analysis results of oracle.analyze_batch (or of the device):
  stream header      flac/encoder.py:61-83, 170-189 (magic, STREAMINFO block)
  frame header       flac/encoder.py:194-234 (+ coded_number.py:7-39, crc.py:18-22)
  subframe header    flac/encoder.py:553-569
  fixed / LPC body   flac/encoder.py:581-627 (warm-up, precision, shift, coefficients)
  residual           flac/encoder.py:765-806 (coding method, partition order, parameter,
                     Rice codes: x >> p zeros, a one, the low p bits MSB first)
  padding + CRC-16   flac/encoder.py:159-163 (crc.py:25-31)
Bits are accumulated MSB first in a Python integer (binary.py:168-206 writes the same
bits one byte at a time); Rice codes are packed with numpy.

Pinned by the reference's own encode() output: tests/test_frame_writer_golden.py
rebuilds the golden stream hashes of tests/golden/streams.json from the oracle
analysis + this writer.
"""
import numpy as np

KIND_LPC = 1
BLOCK_SIZE_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11,
                    4096: 12, 8192: 13, 16384: 14, 32768: 15}
_EXC = {1: ZeroDivisionError, 2: AssertionError, 3: ValueError, 4: OverflowError}


class Bits:
    """MSB-first bit accumulator (the bit order of binary.Put)."""

    def __init__(self):
        self.v = 0
        self.n = 0

    def put(self, x: int, width: int):
        if width:
            self.v = (self.v << width) | (int(x) & ((1 << width) - 1))
            self.n += width

    def put_packed(self, packed: bytes, nbits: int):
        if nbits:
            self.put(int.from_bytes(packed, "big") >> (8 * len(packed) - nbits), nbits)

    def to_bytes(self) -> bytes:
        assert self.n % 8 == 0
        return self.v.to_bytes(self.n // 8, "big")


def crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


_CRC16 = []
for _v in range(256):
    _r = _v << 8
    for _ in range(8):
        _r = ((_r << 1) ^ 0x8005) & 0xFFFF if _r & 0x8000 else (_r << 1) & 0xFFFF
    _CRC16.append(_r)


def crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c = ((c << 8) & 0xFFFF) ^ _CRC16[(c >> 8) ^ b]
    return c


def coded_number(x: int) -> bytes:
    """coded_number.py:7-39."""
    n = x.bit_length()
    for size, bits in ((1, 7), (2, 11), (3, 16), (4, 21), (5, 26), (6, 31)):
        if n <= bits:
            break
    else:
        raise ValueError(f"Cannot encode coded number: {x}")
    if size == 1:
        return bytes([x])
    groups = [(x >> (6 * i)) & 0x3F for i in reversed(range(size))]
    return bytes([(((1 << size) - 1) << (8 - size)) | groups[0]] + [0x80 | g for g in groups[1:]])


def stream_header(sample_rate: int, sample_size: int, channels: int, frames: int, block_size: int) -> bytes:
    """fLaC + last-block STREAMINFO header + STREAMINFO (md5 zeros, frame sizes 0)."""
    b = Bits()
    for v, w in ((block_size, 16), (block_size, 16), (0, 24), (0, 24), (sample_rate, 20), (channels - 1, 3),
                 (sample_size - 1, 5), (frames, 36)):
        b.put(v, w)
    return b"fLaC" + bytes([0x80, 0, 0, 34]) + b.to_bytes() + bytes(16)


def frame_header(index: int, block_size: int) -> bytes:
    """encode()'s frame header: fixed blocking, rate/size from STREAMINFO, channels L_R."""
    code = BLOCK_SIZE_CODES.get(block_size)
    if code is None:
        bl = block_size.bit_length()
        code = 6 if bl <= 8 else 7 if bl <= 16 else None
        if code is None:
            raise ValueError(f"Cannot encode block size: {block_size}")
    h = bytearray([0xFF, 0xF8, code << 4, 0x10]) + coded_number(index)
    if code == 6:
        h += bytes([block_size - 1])
    elif code == 7:
        h += (block_size - 1).to_bytes(2, "big")
    h.append(crc8(bytes(h)))
    return bytes(h)


def rice_packed(values, params) -> tuple:
    """Rice codes (put_rice_int, encoder.py:798-806) of zig-zag values with per-value
    parameters, as (MSB-first packed bytes, bit count)."""
    x = np.asarray(values, dtype=np.uint64)
    p = np.asarray(params, dtype=np.int64)
    q = (x >> p.astype(np.uint64)).astype(np.int64)
    width = q + 1 + p
    ends = np.cumsum(width)
    total = int(ends[-1]) if len(ends) else 0
    one = ends - width + q
    bitmap = np.zeros(total, dtype=np.uint8)
    bitmap[one] = 1
    for b in range(int(p.max()) if len(p) else 0):
        sel = p > b
        shift = (p[sel] - 1 - b).astype(np.uint64)
        bitmap[one[sel] + 1 + b] = ((x[sel] >> shift) & np.uint64(1)).astype(np.uint8)
    return np.packbits(bitmap).tobytes(), total


def subframe(bits: Bits, samples, m, zz, params, n: int, sample_size: int, precision: int):
    """One subframe from a unit's analysis result m (flacmi_unit_meta fields)."""
    order = int(m["order"])
    lpc = int(m["kind"]) == KIND_LPC
    bits.put(0, 1)
    bits.put((0b100000 | (order - 1)) if lpc else (0b001000 | order), 6)
    bits.put(0, 1)
    for s in samples[:order]:
        bits.put(int(s), sample_size)
    if lpc:
        if precision - 1 == 0b1111:
            raise AssertionError()
        bits.put(precision - 1, 4)
        bits.put(int(m["shift"]), 5)
        for c in m["coefs"][: int(m["ncoefs"])]:
            bits.put(int(c), precision)
    method = int(m["coding_method"])
    po = int(m["part_order"])
    bits.put(0b00 if method == 4 else 0b01, 2)
    bits.put(po, 4)
    ps = n >> po
    lens = [ps - order] + [ps] * ((1 << po) - 1)
    pos = 0
    for prm, ln in zip(params, lens):
        bits.put(int(prm), method)
        packed, nb = rice_packed(zz[pos:pos + ln], np.full(ln, int(prm), dtype=np.int64))
        bits.put_packed(packed, nb)
        pos += ln


def frame(index: int, n: int, rows, metas, zz_rows, params_rows, sample_size: int, precision: int) -> bytes:
    """One frame: channel c is rows[c] / metas[c]; zz_rows[c] is the chosen residual
    (res_len zig-zag values); params_rows[c] the n_parts Rice parameters.  Raises the
    reference's exception where the reference would (header, analysis, writer)."""
    bits = Bits()
    for b in frame_header(index, n):
        bits.put(b, 8)
    for c in range(len(rows)):
        st = int(metas[c]["status"])
        if st != 0:
            raise _EXC.get(st, RuntimeError)()
        subframe(bits, rows[c], metas[c], zz_rows[c], params_rows[c], n, sample_size, precision)
    bits.put(0, (8 - bits.n % 8) % 8)
    body = bits.to_bytes()
    return body + crc16(body).to_bytes(2, "big")


def frames_from_analysis(rows: np.ndarray, out: dict, channels: int, block_len: int, tail_len: int,
                         sample_size: int, precision: int, first_frame: int = 0) -> list:
    """Frames of a batch from analyze results (oracle.analyze_batch or the device's
    analyze(): meta, rice_params and residual rows with the chosen residual at
    [res_offset, res_offset + res_len)).  Frame f = rows [f*channels, (f+1)*channels).
    A frame the reference fails on is returned as the exception instance."""
    nf = rows.shape[0] // channels
    frames = []
    for f in range(nf):
        n = tail_len if (f == nf - 1 and tail_len) else block_len
        us = range(f * channels, (f + 1) * channels)
        metas = [out["meta"][u] for u in us]
        zz = [out["residual"][u][int(m["res_offset"]):int(m["res_offset"]) + int(m["res_len"])]
              for u, m in zip(us, metas)]
        prm = [out["rice_params"][u][: int(m["n_parts"])] for u, m in zip(us, metas)]
        try:
            frames.append(frame(first_frame + f, n, [rows[u] for u in us], metas, zz, prm, sample_size,
                                precision))
        except (ValueError, AssertionError, ZeroDivisionError, OverflowError) as e:
            frames.append(e)
    return frames
