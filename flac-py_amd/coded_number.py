"""FLAC's UTF-8-like frame/sample number coding (flac/coded_number.py semantics)."""


def required_bytes(x: int) -> int:
    n = x.bit_length()
    for size, bits in ((1, 7), (2, 11), (3, 16), (4, 21), (5, 26), (6, 31)):
        if n <= bits:
            return size
    raise ValueError(f"Cannot encode coded number: {x}")


def encode(x: int) -> bytes:
    assert 0 <= x.bit_length() <= 36
    size = required_bytes(x)
    if size == 1:
        return bytes([x])
    tail = [0x80 | ((x >> (6 * i)) & 0x3F) for i in range(size - 2, -1, -1)]
    lead = ((0xFF << (8 - size)) & 0xFF) | (x >> (6 * (size - 1)))
    return bytes([lead] + tail)


def following_bytes(b0: int) -> int:
    for count, prefix in ((6, 0xFE), (5, 0xFC), (4, 0xF8), (3, 0xF0), (2, 0xE0), (1, 0xC0)):
        if b0 >= prefix:
            return count
    return 0


def decode(bs: bytes) -> int:
    size = following_bytes(bs[0]) + 1
    assert size == len(bs)
    if size == 1:
        return bs[0]
    x = bs[0] & (0x7F >> size)
    for b in bs[1:]:
        x = (x << 6) | (b & 0x3F)
    return x
