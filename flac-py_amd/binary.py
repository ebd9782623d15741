"""MSB-first bit writer/reader with the interface of flac/binary.py (mask :6-17,
extract :20-30, Get :78-141, Put :144-216).

Put accumulates bits in a Python integer and flushes whole bytes, and can append a
pre-packed bit string (`bits`) in one step — the Rice codes of a residual are packed
with numpy (`rice_bits`) instead of one `uint` call per bit.
"""
from io import BytesIO

import numpy as np


def mask(n: int) -> int:
    return (1 << n) - 1


def extract(x: int, size: int, start: int, stop: int) -> int:
    """Bits [start, stop) of the size-bit field x, counted from the MSB."""
    return (x >> (size - stop)) & mask(stop - start)


class _Bits:
    def __init__(self):
        self._bit_offset = 0

    @property
    def is_aligned(self) -> bool:
        return self._bit_offset == 0

    @property
    def bit_offset(self) -> int:
        return self._bit_offset

    @property
    def bits_until_alignment(self) -> int:
        return (8 - self._bit_offset) % 8


class Put(_Bits):
    def __init__(self):
        super().__init__()
        self._out = bytearray()
        self._acc = 0  # pending bits, fewer than 8, right-aligned

    def uint(self, x: int, n: int):
        """Append the low n bits of x (two's complement for negative x), MSB first."""
        if n == 0:
            return
        acc = (self._acc << n) | (x & mask(n))
        total = self._bit_offset + n
        keep = total & 7
        nbytes = total >> 3
        if nbytes:
            self._out += (acc >> keep).to_bytes(nbytes, "big")
            acc &= mask(keep)
        self._acc = acc
        self._bit_offset = keep

    def bool(self, x: bool):
        self.uint(1 if x is True else 0, 1)

    def bytes(self, bs: bytes):
        assert self._bit_offset == 0
        self._out += bs

    def bits(self, packed: bytes, nbits: int):
        """Append the first nbits of an MSB-first packed bit string."""
        if nbits <= 0:
            return
        if self._bit_offset == 0 and nbits % 8 == 0:
            self._out += packed[: nbits // 8]
            return
        v = int.from_bytes(packed, "big") >> (8 * len(packed) - nbits)
        self.uint(v, nbits)

    @property
    def buffer(self) -> bytes:
        assert self.is_aligned is True
        return bytes(self._out)


def rice_bits(values: np.ndarray, params: np.ndarray) -> tuple:
    """Rice codes of zig-zag values (encoder.py:798-806 per value: x >> p zeros, a one, the
    low p bits MSB first) for per-value parameters, as (packed bytes, bit count)."""
    x = np.asarray(values, dtype=np.uint64)
    p = np.asarray(params, dtype=np.int64)
    q = (x >> p.astype(np.uint64)).astype(np.int64)
    width = q + 1 + p
    ends = np.cumsum(width)
    total = int(ends[-1]) if len(ends) else 0
    starts = ends - width
    bitmap = np.zeros(total, dtype=np.uint8)
    one = starts + q
    bitmap[one] = 1
    pmax = int(p.max()) if len(p) else 0
    for b in range(pmax):  # data bit b (from the MSB side) of every value with p > b
        sel = p > b
        shift = (p[sel] - 1 - b).astype(np.uint64)
        bitmap[one[sel] + 1 + b] = ((x[sel] >> shift) & np.uint64(1)).astype(np.uint8)
    return np.packbits(bitmap).tobytes(), total


class Get(_Bits):
    def __init__(self, buffer):
        super().__init__()
        self._buffer = buffer if hasattr(buffer, "read") else BytesIO(buffer)
        self._cur = 0

    def _byte(self) -> int:
        b = self._buffer.read(1)
        if len(b) != 1:
            raise EOFError()
        return b[0]

    def uint(self, n: int) -> int:
        x = 0
        while n > 0:
            if self._bit_offset == 0:
                self._cur = self._byte()
            take = min(n, 8 - self._bit_offset)
            x = (x << take) | extract(self._cur, 8, self._bit_offset, self._bit_offset + take)
            self._bit_offset = (self._bit_offset + take) & 7
            n -= take
        return x

    def sint(self, n: int) -> int:
        x = self.uint(n)
        return x - ((x >> (n - 1)) << n)

    def bool(self) -> bool:
        return self.uint(1) == 1

    def bytes(self, n: int) -> bytes:
        assert self._bit_offset == 0
        bs = self._buffer.read(n)
        if n < 1:
            raise ValueError("n must be greater than zero.")
        if len(bs) != n:
            raise EOFError()
        return bs
