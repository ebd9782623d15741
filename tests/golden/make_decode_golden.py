"""Golden fixtures for the device decoder verifier (csrc/k_decode.hip), produced by the
reference's own frame decoder.

Run ONLY in the build container, where the reference is readable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_decode_golden.py

flac-py's encoder only ever writes FIXED / LPC subframes in independent-channel frames,
so the frames here are assembled bit by bit by this script (its own writer, below) to
cover everything the reference decoder reads: CONSTANT / VERBATIM subframes, wasted-bits
flags, escaped and Rice5Bit partitions, L_S / S_R / M_S stereo, uncommon block sizes and
sample rates, 1..7-byte coded numbers, 24- and 32-bit samples, LPC orders up to 32, and one
malformed frame per assertion / exception of the decoder.  Each frame is then read back by
the reference (flac.decoder.get_frame + decode_frame, decoder.py:111-130, :431-498 --
imported read-only from /root/reference) and the fixture records its decoded samples or
the exception class it raised.  The GPU box never runs this script.
"""
import hashlib
import io
import json
import os
import random
import sys

REF = os.environ.get("FLAC_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from flac import decoder as D  # noqa: E402  (the reference, imported read-only)
from flac.binary import Get  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
FIXED = ((), (1,), (2, -1), (3, -3, 1), (4, -6, 4, -1))


class Bits:
    """MSB-first bit writer (this script's own)."""

    def __init__(self):
        self.v, self.n = 0, 0

    def u(self, x, n):
        assert 0 <= x < (1 << n) or n == 0
        self.v, self.n = (self.v << n) | x, self.n + n

    def s(self, x, n):
        assert -(1 << (n - 1)) <= x < (1 << (n - 1))
        self.u(x & ((1 << n) - 1), n)

    def rice(self, x, p):
        z = (x << 1) ^ (x >> 63) if x >= 0 else ((-x) << 1) - 1
        self.u(0, z >> p)
        self.u(1, 1)
        self.u(z & ((1 << p) - 1), p)

    def pad(self):
        if self.n % 8:
            self.u(0, 8 - self.n % 8)

    def data(self):
        assert self.n % 8 == 0
        return self.v.to_bytes(self.n // 8, "big") if self.n else b""


def crc8(bs):
    c = 0
    for b in bs:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(bs):
    c = 0
    for b in bs:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def coded(x):
    if x < 128:
        return bytes([x])
    n = 2
    while x >= (1 << (5 * n + 1)):
        n += 1
    out = [(0x80 | (x >> (6 * i)) & 0x3F) for i in reversed(range(n - 1))]
    return bytes([((0xFF << (8 - n)) & 0xFF) | (x >> (6 * (n - 1)))] + out)


def header(bs_code, bs, sr_code=0, ch_code=0, ss_code=0, fno=0, sync=0x7FFC, reserved=0, sr_extra=None):
    b = Bits()
    b.u(sync, 15)
    b.u(0, 1)
    b.u(bs_code, 4)
    b.u(sr_code, 4)
    b.u(ch_code, 4)
    b.u(ss_code, 3)
    b.u(reserved, 1)
    for byte in coded(fno):
        b.u(byte, 8)
    if bs_code == 6:
        b.u(bs - 1, 8)
    elif bs_code == 7:
        b.u(bs - 1, 16)
    if sr_code == 12:
        b.u(sr_extra or 48, 8)
    elif sr_code in (13, 14):
        b.u(sr_extra or 4410, 16)
    h = b.data()
    return h + bytes([crc8(h)])


def predict(x, coefs, shift, order):
    return [x[i] - (sum(c * x[i - 1 - j] for j, c in enumerate(coefs)) >> shift) for i in range(order, len(x))]


def residual_bits(b, r, bs, order, po, params, method=0, esc=None):
    """Rice partitions of residual r (len bs - order); params per partition; esc: {k: bits}."""
    b.u(method, 2)
    b.u(po, 4)
    plen = bs >> po
    i = 0
    pb = 5 if method else 4
    for k in range(1 << po):
        n = plen - order if k == 0 else plen
        part = r[i:i + n]
        i += n
        if esc and k in esc:
            b.u((1 << pb) - 1, pb)
            b.u(esc[k], 5)
            for x in part:
                b.s(x, esc[k]) if esc[k] else None
        else:
            # the listed parameter is a lower bound: raised to the encoder's own choice
            # floor(log2(mean zig-zag)) so no code gets a huge unary part
            zz = [2 * v if v >= 0 else -2 * v - 1 for v in part]
            mean = sum(zz) // max(len(zz), 1)
            p = max(params[k], mean.bit_length() - 1 if mean >= 1 else 0)
            assert p < (1 << pb) - 1
            b.u(p, pb)
            for x in part:
                b.rice(x, p)


def sub_fixed(b, x, order, ss, po, params, method=0, esc=None, wasted=0, pad=0):
    b.u(pad, 1)
    b.u(8 | order, 6)
    if wasted:
        b.u(1, 1)  # get_wasted_bits (decoder.py:346-355) returns the count of zeros that follow
        b.u(0, wasted)
        b.u(1, 1)
    else:
        b.u(0, 1)
    w = ss - wasted
    for v in x[:order]:
        b.s(v, w)
    residual_bits(b, predict(x, FIXED[order], 0, order), len(x), order, po, params, method, esc)


def sub_lpc(b, x, coefs, prec, shift, ss, po, params, method=0, esc=None, prec_field=None, raw_resid=None):
    order = len(coefs)
    b.u(0, 1)
    b.u(32 | (order - 1), 6)
    b.u(0, 1)
    for v in x[:order]:
        b.s(v, ss)
    b.u(prec - 1 if prec_field is None else prec_field, 4)
    b.s(shift, 5)
    for c in coefs:
        b.s(c, prec)
    r = raw_resid if raw_resid is not None else predict(x, coefs, shift, order)
    residual_bits(b, r, len(x), order, po, params, method, esc)


def frame(hdr, subs):
    b = Bits()
    for byte in hdr:
        b.u(byte, 8)
    for f in subs:
        f(b)
    b.pad()
    d = b.data()
    return d + crc16(d).to_bytes(2, "big")


def signal(rng, n, bits, tones=2):
    import math
    amp = (1 << (bits - 1)) - 1
    ph = [rng.random() * 6.28 for _ in range(tones)]
    fr = [rng.uniform(0.001, 0.05) for _ in range(tones)]
    out = []
    for i in range(n):
        v = sum(0.3 * math.sin(ph[t] + 6.283 * fr[t] * i) for t in range(tones)) + rng.gauss(0, 0.01)
        out.append(max(-amp - 1, min(amp, int(round(v * amp)))))
    return out


def lpc_coefs(rng, order, prec):
    # a stable-ish predictor: binomial-like smoothing weights scaled to the precision
    base = FIXED[min(order, 2)] + (0,) * max(0, order - 2)
    lim = (1 << (prec - 1)) - 1
    shift = prec - 4
    return [max(-lim - 1, min(lim, int(c * (1 << shift)) + rng.randint(-3, 3))) for c in base], shift


def build():
    rng = random.Random(20261016)
    cases = []

    def add(name, data, channels, ss, site=None, expect_verify=None, truncate=None):
        cases.append({"name": name, "data": data, "channels": channels, "ss": ss, "site": site,
                      "verify": expect_verify, "truncate": truncate})

    # --- valid frames --------------------------------------------------------------
    add("constant_192", frame(header(1, 192, ch_code=0, ss_code=4, fno=3),
                              [lambda b: (b.u(0, 1), b.u(0, 6), b.u(0, 1), b.s(-1234, 16))]), 1, 16)
    vb = [rng.randint(-32768, 32767) for _ in range(256)]
    add("verbatim_256", frame(header(8, 256, ch_code=0, ss_code=4, fno=200),
                              [lambda b: (b.u(0, 1), b.u(1, 6), b.u(0, 1), [b.s(v, 16) for v in vb])]), 1, 16)
    for o in range(5):
        x = signal(rng, 576, 16)
        add(f"fixed{o}_576", frame(header(2, 576, ch_code=0, ss_code=0, fno=1000 + o),
                                   [lambda b, x=x, o=o: sub_fixed(b, x, o, 16, 2, [3, 5, 7, 9])]), 1, 16)
    x = signal(rng, 1152, 16)
    add("fixed2_wasted2", frame(header(3, 1152, ch_code=0, ss_code=4, fno=5),
                                [lambda b: sub_fixed(b, [v >> 2 for v in x], 2, 16, 0, [6], wasted=2)]), 1, 16)
    for order, prec in ((1, 5), (8, 12), (12, 15), (32, 15)):
        x = signal(rng, 1024, 24 if order == 32 else 16, 3)
        c, sh = lpc_coefs(rng, order, prec)
        ss = 24 if order == 32 else 16
        add(f"lpc{order}_p{prec}", frame(header(10, 1024, ch_code=0, ss_code=6 if ss == 24 else 4, fno=70000 + order),
                                         [lambda b, x=x, c=c, sh=sh, prec=prec, ss=ss:
                                          sub_lpc(b, x, c, prec, sh, ss, 3, [0, 1, 2, 3, 4, 5, 6, 7],
                                                  method=int(ss > 16))]), 1, ss)
    x = [rng.randint(-3, 3) for _ in range(256)]
    add("fixed1_quiet_p0", frame(header(8, 256, ch_code=0, ss_code=4, fno=11),
                                 [lambda b: sub_fixed(b, x, 1, 16, 2, [0, 0, 0, 0])]), 1, 16)
    x = signal(rng, 1000, 20)
    c, sh = lpc_coefs(rng, 6, 14)
    add("lpc6_rice5_escape_bs16", frame(header(7, 1000, sr_code=13, ch_code=0, ss_code=5, fno=(1 << 26) + 9),
                                        [lambda b: sub_lpc(b, x, c, 14, sh, 20, 3, [15, 16, 0, 20, 17, 18, 19, 22],
                                                           method=1, esc={2: 21})]), 1, 20)
    x = signal(rng, 200, 8)
    add("fixed1_escape_bs8", frame(header(6, 200, sr_code=12, ch_code=0, ss_code=1, fno=(1 << 31) - 1),
                                   [lambda b: sub_fixed(b, x, 1, 8, 1, [2, 3], esc={0: 9})]), 1, 8)
    x = signal(rng, 512, 32)
    add("fixed3_32bit", frame(header(9, 512, sr_code=14, ch_code=0, ss_code=7, fno=127),
                              [lambda b: sub_fixed(b, x, 3, 32, 1, [27, 28], method=1)]), 1, 32)
    for code, nm in ((8, "L_S"), (9, "S_R"), (10, "M_S")):
        L = signal(rng, 576, 16)
        R = [v + rng.randint(-500, 500) for v in L]
        R = [max(-32768, min(32767, v)) for v in R]
        if code == 8:
            ch = [L, [a - b for a, b in zip(L, R)]]
        elif code == 9:
            ch = [[a - b for a, b in zip(L, R)], R]
        else:
            ch = [[(a + b) >> 1 for a, b in zip(L, R)], [a - b for a, b in zip(L, R)]]
        ssz = [16 + (code == 9), 16 + (code != 9)]
        add(f"stereo_{nm}", frame(header(2, 576, ch_code=code, ss_code=4, fno=77),
                                  [lambda b, s=ch[0], w=ssz[0]: sub_fixed(b, s, 2, w, 1, [9, 10]),
                                   lambda b, s=ch[1], w=ssz[1]: sub_fixed(b, s, 1, w, 1, [9, 10])]), 2, 16)
    x0, x1 = signal(rng, 4608, 16), signal(rng, 4608, 16)
    add("stereo_L_R_4608", frame(header(5, 4608, ch_code=1, ss_code=4, fno=4000),
                                 [lambda b: sub_fixed(b, x0, 2, 16, 5, [8] * 32),
                                  lambda b: sub_fixed(b, x1, 4, 16, 0, [9])]), 2, 16)
    bad = bytearray(cases[2]["data"])
    bad[-1] ^= 0x5A
    add("bad_crc16", bytes(bad), 1, 16, expect_verify="crc16")

    # --- malformed frames: one per assertion / exception of the reference decoder ---
    x = signal(rng, 576, 16)
    ok_sub = [lambda b: sub_fixed(b, x, 2, 16, 1, [7, 8])]
    add("err_sync", frame(header(2, 576, sync=0x7FFD), ok_sub), 1, 16, site="sync")
    add("err_bs_code0", frame(header(0, 576), ok_sub), 1, 16, site="block_size_code")
    add("err_sr_code15", frame(header(2, 576, sr_code=15), ok_sub), 1, 16, site="sample_rate_code")
    add("err_ch_code11", frame(header(2, 576, ch_code=11), ok_sub), 1, 16, site="channels_code")
    add("err_ss_code3", frame(header(2, 576, ss_code=3), ok_sub), 1, 16, site="sample_size_code")
    add("err_reserved", frame(header(2, 576, reserved=1), ok_sub), 1, 16, site="reserved")
    add("err_subframe_pad", frame(header(2, 576), [lambda b: sub_fixed(b, x, 2, 16, 1, [7, 8], pad=1)]), 1, 16,
        site="subframe_pad")
    add("err_subframe_type", frame(header(2, 576), [lambda b: (b.u(0, 1), b.u(2, 6), b.u(0, 1), b.u(0, 64))]), 1, 16,
        site="subframe_type")
    c, sh = lpc_coefs(rng, 4, 8)
    add("err_lpc_precision", frame(header(2, 576), [lambda b: sub_lpc(b, x, c, 8, sh, 16, 0, [9], prec_field=15)]),
        1, 16, site="lpc_precision")
    add("err_coding_method", frame(header(2, 576), [lambda b: (b.u(0, 1), b.u(9, 6), b.u(0, 1), b.s(x[0], 16),
                                                               b.u(2, 2), b.u(0, 64))]), 1, 16, site="coding_method")
    add("err_partitions", frame(header(7, 1000), [lambda b: (b.u(0, 1), b.u(9, 6), b.u(0, 1), b.s(x[0], 16),
                                                             b.u(0, 2), b.u(4, 4), b.u(0, 64))]), 1, 16,
        site="partitions")
    add("err_escape_zero", frame(header(2, 576), [lambda b: sub_fixed(b, x, 2, 16, 1, [7, 8], esc={1: 0})]), 1, 16,
        site="escape_zero")
    add("err_neg_shift", frame(header(2, 576), [lambda b: sub_lpc(b, x, [1, 0], 6, -2, 16, 0, [12],
                                                                  raw_resid=[0] * 574)]), 1, 16, site="neg_shift")
    good = cases[2]["data"]
    # a frame whose last data byte ends with padding bits: set them (CRC recomputed)
    while True:
        b = Bits()
        for byte in header(2, 576):
            b.u(byte, 8)
        sub_fixed(b, x, 2, 16, 1, [7, 8])
        padbits = (8 - b.n % 8) % 8
        if padbits:
            break
        x = signal(rng, 576, 16)
    b.u(1, padbits)
    d = b.data()
    add("err_padding", d + crc16(d).to_bytes(2, "big"), 1, 16, site="padding")
    add("err_eof", good[: len(good) // 2], 1, 16, site="eof")

    out = []
    for cs in cases:
        data = cs["data"]
        try:
            get = Get(io.BytesIO(data))
            fr = D.get_frame(get, cs["ss"])
            dec = D.decode_frame(fr)
            flat = b"".join(int(v).to_bytes(8, "little", signed=True) for ch in dec for v in ch)
            res = {"decoded_sha256": hashlib.sha256(flat).hexdigest(), "decoded_head": [ch[:8] for ch in dec],
                   "exception": None, "block_size": fr.header.block_size,
                   "header_channels": fr.header.channels.count}
        except Exception as e:  # noqa: BLE001  -- the reference's exception class is the fixture
            res = {"decoded_sha256": None, "exception": type(e).__name__}
        out.append({"name": cs["name"], "hex": data.hex(), "channels": cs["channels"], "sample_size": cs["ss"],
                    "site": cs["site"], "verify": cs["verify"], **res})
        print(f"{cs['name']:28s} {len(data):6d} B  -> {res['exception'] or 'ok'}")
    with open(os.path.join(OUT, "decode.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_decode_golden.py", "reference": "flac.decoder.get_frame + "
                   "decode_frame (decoder.py:111-130, :431-498)", "cases": out}, f, separators=(",", ":"))


if __name__ == "__main__":
    build()
