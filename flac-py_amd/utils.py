"""Small helpers with the semantics of flac/utils.py (argparse_range :12-28, batch :31-40,
clamp :43-48, group :61-66, log2i :73-80, zigzag :87-94)."""
from itertools import islice
from typing import Iterator, TypeVar

T = TypeVar("T")


def argparse_range(s: str) -> range:
    """'N' -> range(0, N+1); 'M,N' -> range(M, N+1) (M < N required)."""
    parts = [int(p) for p in s.split(",")]
    assert 1 <= len(parts) <= 2
    assert all(a < b for a, b in zip(parts, parts[1:]))
    return range(parts[0], parts[1] + 1) if len(parts) == 2 else range(0, parts[0] + 1)


def batch(it: Iterator[T], n: int) -> Iterator[list]:
    """Consecutive lists of n items; the last one may be shorter."""
    if n < 1:
        raise ValueError("n must be greater than zero")
    it = iter(it)
    while True:
        chunk = list(islice(it, n))
        if not chunk:
            return
        yield chunk


def clamp(x: int, lo: int, hi: int) -> int:
    return lo if x < lo else hi if x > hi else x


def group(xs, n):
    return [xs[i:i + n] for i in range(0, len(xs), n)]


def log2i(x: int) -> int:
    assert x > 0
    return x.bit_length() - 1


def zigzag_encode(x: int) -> int:
    assert -(1 << 63) < x < (1 << 64) - 1
    return (x << 1) if x >= 0 else ((-x) << 1) - 1


def zigzag_decode(x: int) -> int:
    return (x >> 1) if not (x & 1) else -((x + 1) >> 1)
