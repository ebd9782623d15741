"""MSB-first bit writer/reader with the interface of flac/binary.py (mask :6-17,
extract :20-30, Get :78-141, Put :144-216).

Put accumulates bits in a Python integer and flushes whole bytes.  It writes only the
stream header here: frames (Rice codes, headers, CRCs) are written on the device
(csrc/k_frame.hip).
"""
from io import BytesIO


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

    @property
    def buffer(self) -> bytes:
        assert self.is_aligned is True
        return bytes(self._out)


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
