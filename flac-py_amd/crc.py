"""CRC-8 (x^8+x^2+x+1) and CRC-16 (x^16+x^15+x^2+1), MSB-first, init 0, as used by FLAC
frame headers/footers (flac/crc.py, polynomials flac/common.py:12-13)."""
from functools import lru_cache


@lru_cache(maxsize=None)
def _table(width: int, poly: int) -> tuple:
    top = 1 << (width - 1)
    mask = (1 << width) - 1
    out = []
    for byte in range(256):
        r = byte << (width - 8)
        for _ in range(8):
            r = ((r << 1) ^ poly) if (r & top) else (r << 1)
        out.append(r & mask)
    return tuple(out)


def crc8(data: bytes, generator: int, initial_value: int = 0) -> int:
    t = _table(8, generator & 0xFF)
    c = initial_value
    for b in data:
        c = t[c ^ b]
    return c


def crc16(data: bytes, generator: int, initial_value: int = 0) -> int:
    t = _table(16, generator & 0xFFFF)
    c = initial_value
    for b in data:
        c = ((c << 8) & 0xFFFF) ^ t[(c >> 8) ^ b]
    return c
