/* k_decode.hip — the FLAC frame decoder on the device, used as the round-trip verifier of
 * the encode path (BASELINE config 5).
 *
 * The reference decodes one frame at a time on the host, one bit at a time through
 * binary.Get (decoder.py:111-130 get_frame, :133-245 the header, :267-355 subframes,
 * :358-421 the residual, :431-498 sample restoration).  Every step inside a frame is
 * sequential: Rice codes are variable-length with no partition index in the stream, and
 * sample restoration is a linear recurrence (each sample needs the `order` restored
 * samples before it).  Frames, however, are independent and their byte offsets are known
 * (the writer's scan produced them), so:
 *
 *   k_decode_fx  one LANE per frame, 256 frames per workgroup, for the frames every check
 *              passes and whose subframes are CONSTANT, VERBATIM or FIXED (what the encoder
 *              writes for almost every block: flac-py's negated LPC predictor rarely wins).
 *              A FIXED sample is restored by four wrapping 32-bit adds (the order-k
 *              predictor inverted as k running differences), a Rice code whose unary run
 *              and low bits lie inside the 32-bit window by one v_ffbh, one shift-add and no
 *              64-bit arithmetic; partition headers, escapes, long codes and the stream's
 *              last dwords take a divergent general branch.  Decoded samples go through a
 *              16-slot LDS ring per lane and are compared with the source rows every 16.
 *              Any check that fails, an LPC subframe, wasted bits, stereo decorrelation or a
 *              sample mismatch makes the lane hand its frame to the list below instead:
 *              this kernel only ever reports status 0.
 *   k_decode   one LANE per listed frame (or per frame, knob FLACMI_DECODE_GENERIC): the
 *              general decoder with every check and the exact status precedence.  Sample
 *              i of every lane's subframe is restored in loop iteration i, so the lanes of a
 *              wave stay in lock-step and the per-lane history ring in LDS (32 slots x 64
 *              lanes, slot-major: a lane's column is one bank) is conflict-free.  Every 32
 *              samples a lane flushes its ring column as 128 contiguous bytes of its decoded
 *              row and compares them with the source row.
 *   Both read the frame with a 64-bit big-endian bit window refilled one dword at a time
 *   (frames start at any byte) and fold the CRC-16 as whole dwords leave the window, with
 *   the writer's slice-by-4 table (the reference reads CRC-8 / CRC-16 unchecked).
 *   k_decorr   frames whose header selects L_S / S_R / M_S stereo (flac-py's encoder never
 *              writes them) are recombined in place (decoder.py:431-448) and compared here,
 *              one workgroup per frame.
 *
 * Status precedence: the first exception the reference decoder would raise wins over any
 * verifier finding; among verifier findings the first one found is kept. */
#include "device_common.h"

namespace flacmi {

constexpr int kDecThreads = 64; /* one wave per workgroup: lanes are independent frames */
constexpr int kRingSlots = 32;  /* LPC order <= 32 */

enum : int32_t {
    DS_SYNC = FLACMI_DSITE_SYNC, DS_BS_CODE, DS_SR_CODE, DS_CH_CODE, DS_SS_CODE, DS_RESERVED,
    DS_SUB_PAD, DS_SUB_TYPE, DS_LPC_PREC, DS_CODING, DS_PARTS, DS_ESC_ZERO, DS_NEG_SHIFT,
    DS_PADDING, DS_EOF, DS_CRC8, DS_CRC16, DS_FRAME_END, DS_FRAME_NO, DS_BLOCK_SIZE, DS_CHANNELS,
    DS_SAMPLES,
};
static_assert(DS_SAMPLES == FLACMI_DSITE_SAMPLES, "flacmi_decode_site order");

__device__ __forceinline__ int32_t dstat(int32_t site) {
    int32_t s;
    if (site == DS_EOF) s = FLACMI_STATUS_EOF;
    else if (site == DS_CODING || site == DS_ESC_ZERO || site == DS_NEG_SHIFT) s = FLACMI_STATUS_VALUE_ERROR;
    else if (site >= DS_CRC8) s = FLACMI_STATUS_VERIFY;
    else s = FLACMI_STATUS_ASSERTION;
    return (site << 16) | s;
}
__device__ __forceinline__ bool is_ref_error(int32_t st) { return st != 0 && (st & 0xFFFF) != FLACMI_STATUS_VERIFY; }

/* FIXED_PREDICTOR_COEFFICIENTS[o][k] (common.py:15-21): (-1)^k * C(o, k+1) */
__device__ __forceinline__ int32_t fixed_coef(int o, int k) {
    switch (o * 4 + k) {
        case 4: return 1;
        case 8: return 2;
        case 9: return -1;
        case 12: return 3;
        case 13: return -3;
        case 14: return 1;
        case 16: return 4;
        case 17: return -6;
        case 18: return 4;
        case 19: return -1;
        default: return 0;
    }
}
/* SAMPLE_SIZE_DECODING (common.py:249-258); code 3 is rejected before */
__device__ __forceinline__ int sample_size_of(int code) {
    switch (code) {
        case 1: return 8;
        case 2: return 12;
        case 4: return 16;
        case 5: return 20;
        case 6: return 24;
        case 7: return 32;
        default: return 0;
    }
}

/* MSB-first reader over the stream: (hi, lo) are dwords b and b + 1 and the read position
 * is 32 b + 32 - sh, sh in [0, 31], so the next 32 bits are one v_alignbit. */
struct BitReader {
    const uint32_t* w;
    int64_t nw;
    int64_t b;
    uint32_t hi, lo;
    int32_t sh;
    int64_t bnear; /* b >= bnear: a 32-bit read could pass the stream's end */
    bool near;
    /* CRC-16 of the frame folded as whole dwords leave the window, in stream order: dword
     * cnext is the next one due, dwords below cend are inside the CRC range (crc16_fused) */
    const uint16_t* ct = nullptr;
    uint32_t crc = 0;
    int64_t cnext = 0, cend = 0;
    __device__ __forceinline__ uint32_t ld(int64_t i) const {
        return (uint64_t)i < (uint64_t)nw ? __builtin_bswap32(w[i]) : 0u;
    }
    __device__ __forceinline__ void fold(uint32_t be) { /* one whole big-endian dword */
        const uint32_t v = be ^ (crc << 16);
        crc = ct[3 * 256 + (v >> 24)] ^ ct[2 * 256 + ((v >> 16) & 0xFF)] ^ ct[256 + ((v >> 8) & 0xFF)] ^ ct[v & 0xFF];
    }
    __device__ __forceinline__ int64_t pos() const { return 32 * b + 32 - sh; }
    __device__ __forceinline__ void seek(int64_t p, int64_t end_bit) {
        b = (p - 1) >> 5; /* p = 0: dword -1 (reads as 0) */
        sh = (int32_t)(32 * b + 32 - p);
        hi = ld(b);
        lo = ld(b + 1);
        bnear = (end_bit >> 5) - 1;
        near = b >= bnear;
    }
    __device__ __forceinline__ void adv() { /* dword b leaves the window */
        if (ct && b == cnext && b < cend) {
            fold(hi);
            ++cnext;
        }
        hi = lo;
        lo = ld(b + 2);
        ++b;
        near = near || b >= bnear;
    }
    /* the 32 bits at the read position, MSB first */
    __device__ __forceinline__ uint32_t peek32() const { return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh); }
    __device__ __forceinline__ void skip(int n) { /* 0 <= n <= 32 */
        sh -= n;
        if (sh < 0) {
            sh += 32;
            adv();
        }
    }
    __device__ __forceinline__ uint32_t uint(int n) { /* 0 <= n <= 32 (binary.py:97) */
        if (n == 0) return 0;
        const uint32_t v = peek32() >> (32 - n);
        skip(n);
        return v;
    }
    __device__ __forceinline__ uint64_t uint64(int n) { /* 0 <= n <= 64 */
        if (n <= 32) return uint(n);
        const uint64_t hi2 = uint(n - 32);
        return (hi2 << 32) | uint(32);
    }
    /* binary.py:129-131 (n >= 1) */
    __device__ __forceinline__ int64_t sint(int n) {
        const uint64_t x = uint64(n);
        return n >= 64 ? (int64_t)x : (int64_t)(x << (64 - n)) >> (64 - n);
    }
    /* get_rice_int (decoder.py:414-421) followed by zigzag_decode (utils.py); sets eof when
     * the unary run passes `end` (the stream's last bit: the reference raises EOFError). */
    __device__ __forceinline__ int64_t rice(int p, int64_t end, bool& eof) {
        uint64_t q = 0;
        uint32_t W = peek32();
        while (W == 0) {
            q += 32;
            skip(32);
            if (pos() > end) {
                eof = true;
                return 0;
            }
            W = peek32();
        }
        const int z = __builtin_clz(W);
        q += z;
        uint64_t v;
        if (z + 1 + p <= 32) {
            v = (q << p) | (p ? ((W << (z + 1)) >> (32 - p)) : 0u);
            skip(z + 1 + p);
        } else {
            skip(z + 1);
            v = (q << p) | uint(p);
        }
        return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
    }
};

__device__ __forceinline__ int64_t unit_len_d(const DecodeArgs& a, int64_t u) {
    return u >= a.n_units - a.n_tail_units ? a.tail_len : a.block_len;
}

__device__ __forceinline__ int32_t expect_at(const DecodeArgs& a, int64_t u, int64_t i) {
    if (a.expect_bytes == 2) return ((const int16_t*)a.expect)[u * a.expect_stride + i];
    return ((const int32_t*)a.expect)[u * a.expect_stride + i];
}

/* CRC-16 (crc.py:25-31) of stream bytes [b0, b1), continuing from c: slice-by-4 over
 * whole dwords */
__device__ uint32_t crc16_more(const DecodeArgs& a, const uint16_t* t, uint32_t c, int64_t b0, int64_t b1) {
    const uint8_t* bytes = reinterpret_cast<const uint8_t*>(a.words);
    int64_t i = b0;
    for (; i < b1 && (i & 3); ++i) c = ((c << 8) & 0xFFFF) ^ t[((c >> 8) ^ bytes[i]) & 0xFF];
    for (; i + 4 <= b1; i += 4) {
        const uint32_t v = __builtin_bswap32(a.words[i >> 2]) ^ (c << 16);
        c = t[3 * 256 + (v >> 24)] ^ t[2 * 256 + ((v >> 16) & 0xFF)] ^ t[256 + ((v >> 8) & 0xFF)] ^ t[v & 0xFF];
    }
    for (; i < b1; ++i) c = ((c << 8) & 0xFFFF) ^ t[((c >> 8) ^ bytes[i]) & 0xFF];
    return c;
}

/* CRC-16 (crc.py:25-31) of stream bytes [b0, b1): slice-by-4 over whole dwords */
__device__ uint32_t crc16_range(const DecodeArgs& a, const uint16_t* t, int64_t b0, int64_t b1) {
    const uint8_t* bytes = reinterpret_cast<const uint8_t*>(a.words);
    uint32_t c = 0;
    int64_t i = b0;
    for (; i < b1 && (i & 3); ++i) c = ((c << 8) & 0xFFFF) ^ t[((c >> 8) ^ bytes[i]) & 0xFF];
    for (; i + 4 <= b1; i += 4) {
        const uint32_t v = __builtin_bswap32(a.words[i >> 2]) ^ (c << 16);
        c = t[3 * 256 + (v >> 24)] ^ t[2 * 256 + ((v >> 16) & 0xFF)] ^ t[256 + ((v >> 8) & 0xFF)] ^ t[v & 0xFF];
    }
    for (; i < b1; ++i) c = ((c << 8) & 0xFFFF) ^ t[((c >> 8) ^ bytes[i]) & 0xFF];
    return c;
}

/* The general decoder: frame f, every check, the reference's exception precedence. */
__device__ void decode_general(const DecodeArgs& a, const int64_t f, int32_t (*ring)[kDecThreads],
                             int16_t (*coef)[kDecThreads], const uint16_t* crct, const int lane) {
    const int64_t F = a.offsets[f], Fend = a.offsets[f + 1];
    const int64_t end_bit = a.stream_bytes * 8; /* reading past it: EOFError */
    int64_t bad = 0;
    int32_t st = 0;
    auto fail = [&](int32_t site) {
        const int32_t s = dstat(site);
        if (st == 0 || (!is_ref_error(st) && is_ref_error(s))) st = s;
    };
    BitReader g;
    g.w = a.words;
    g.nw = a.n_words;
    /* fused CRC-16 over [F, Fend - 2): the bytes before the first whole dword now, whole
     * dwords as they leave the window, the rest after the footer */
    const int64_t E = Fend - 2;
    const int64_t Fh = (F + 3) & ~(int64_t)3;
    if (a.check_crc && E > F) {
        g.ct = crct;
        g.crc = crc16_more(a, crct, 0u, F, E < Fh ? E : Fh);
        g.cnext = Fh >> 2;
        g.cend = E >> 2;
    }
    g.seek(F * 8, end_bit);
    /* a parse failure after the reader ran off the stream is the EOFError of that read */
    auto pfail = [&](int32_t site) { fail(g.pos() > end_bit ? (int32_t)DS_EOF : site); };

    /* ---- frame header (decoder.py:133-245) ---- */
    int bs = 0, ss = 0, ch_code = 0, nch = 0;
    do {
        if (g.uint(15) != 0x7FFC) { pfail(DS_SYNC); break; }
        (void)g.uint(1); /* blocking strategy */
        const int bcode = g.uint(4);
        if (!(bcode > 0 && bcode < 15)) { pfail(DS_BS_CODE); break; }
        const int rcode = g.uint(4);
        if (rcode == 15) { pfail(DS_SR_CODE); break; }
        ch_code = g.uint(4);
        if (ch_code > 10) { pfail(DS_CH_CODE); break; }
        const int scode = g.uint(3);
        if (scode == 3) { pfail(DS_SS_CODE); break; }
        if (g.uint(1) != 0) { pfail(DS_RESERVED); break; }
        /* coded number (coded_number.py:45-70): lead byte, following_bytes() more, the
         * continuation bytes' low 6 bits (their 10 prefix is not checked) */
        const uint32_t b0 = g.uint(8);
        const int extra = b0 >= 0xFE ? 6 : b0 >= 0xFC ? 5 : b0 >= 0xF8 ? 4 : b0 >= 0xF0 ? 3 : b0 >= 0xE0 ? 2 : b0 >= 0xC0 ? 1 : 0;
        uint64_t fno = extra == 0 ? b0 : (b0 & ((1u << (6 - extra)) - 1));
        for (int k = 0; k < extra; ++k) fno = (fno << 6) | (g.uint(8) & 0x3F);
        if (bcode == 1) bs = 192;
        else if (bcode <= 5) bs = 144 << bcode;
        else if (bcode == 6) bs = (int)g.uint(8) + 1;
        else if (bcode == 7) bs = (int)g.uint(16) + 1;
        else bs = 1 << bcode;
        if (rcode == 12) (void)g.uint(8);
        else if (rcode == 13 || rcode == 14) (void)g.uint(16);
        const int hdr_bytes = (int)((g.pos() >> 3) - F); /* byte-aligned here */
        const uint32_t crc8 = g.uint(8);
        if (g.pos() > end_bit) { pfail(DS_EOF); break; }
        if (a.check_crc) {
            const uint8_t* bytes = reinterpret_cast<const uint8_t*>(a.words);
            uint32_t c = 0; /* x^8 + x^2 + x + 1, init 0 (crc.py:18-22) */
            for (int k = 0; k < hdr_bytes; ++k) {
                c ^= bytes[F + k];
                for (int b = 0; b < 8; ++b) c = (c & 0x80) ? ((c << 1) ^ 0x07) & 0xFF : (c << 1) & 0xFF;
            }
            if (c != crc8) fail(DS_CRC8);
        }
        ss = scode == 0 ? a.sample_size : sample_size_of(scode);
        nch = ch_code <= 7 ? ch_code + 1 : 2;
        /* encoder.py:95 writes L_R whatever the channel count: an L_R frame holds
         * dp->channels subframes (the reference decoder would read two) */
        if (ch_code == 1) nch = a.channels;
        if (nch != a.channels) { pfail(DS_CHANNELS); nch = 0; }
        if (a.first_frame >= 0 && (int64_t)fno != a.first_frame + f) fail(DS_FRAME_NO);
    } while (false);
    if (is_ref_error(st)) nch = 0;
    const bool decorr = ch_code >= 8 && ch_code <= 10;
    if (a.out && bs > a.out_stride) { pfail(DS_BLOCK_SIZE); nch = 0; }
    if (decorr && !a.out) { pfail(DS_CHANNELS); nch = 0; }

    /* ---- subframes (decoder.py:267-421) and their samples (:473-498) ---- */
    bool neg_shift = false;
    for (int c = 0; c < nch; ++c) {
        const int64_t u = f * a.channels + c;
        const bool len_ok = !a.expect || unit_len_d(a, u) == bs;
        if (!len_ok) fail(DS_BLOCK_SIZE);
        const bool cmp = a.expect != nullptr && !decorr && len_ok;
        const bool dbit = (ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1);
        if (g.uint(1) != 0) { pfail(DS_SUB_PAD); break; }
        const int t = g.uint(6);
        if (!(t <= 1 || (t >= 8 && t <= 12) || t >= 32)) { pfail(DS_SUB_TYPE); break; }
        int wasted = 0;
        if (g.uint(1)) { /* get_wasted_bits: count zeros up to a one (parsed, not applied) */
            while (g.uint(1) == 0) {
                ++wasted;
                if (g.pos() > end_bit) break;
            }
        }
        const int w = ss + (dbit ? 1 : 0) - wasted; /* sample_size_ (decoder.py:276) */
        if (w <= 0) { pfail(DS_ESC_ZERO); break; }
        const int order = t >= 32 ? (t & 31) + 1 : t >= 8 ? (t & 7) : 0;
        int64_t cval = 0;
        int shift = 0;
        int pbits = 4;
        int plen = 0;
        if (t == 0) {
            cval = g.sint(w);
        } else if (t >= 8) {
            for (int k = 0; k < order; ++k) ring[k][lane] = (int32_t)g.sint(w); /* warm-up */
            if (t >= 32) {
                const int prec = g.uint(4);
                if (prec == 15) { pfail(DS_LPC_PREC); break; }
                shift = (int)g.sint(5);
                for (int k = 0; k < order; ++k) coef[k][lane] = (int16_t)g.sint(prec + 1);
            } else {
                for (int k = 0; k < order; ++k) coef[k][lane] = (int16_t)fixed_coef(order, k); /* shift 0 */
            }
            const int cm = g.uint(2);
            if (cm > 1) { pfail(DS_CODING); break; }
            pbits = cm ? 5 : 4;
            const int po = g.uint(4);
            if ((bs & ((1 << po) - 1)) != 0 || (bs >> po) <= order) { pfail(DS_PARTS); break; }
            plen = bs >> po;
            /* `>> shift` raises in decode_frame, i.e. only after the whole frame parsed */
            if (order < bs && shift < 0) {
                neg_shift = true;
                shift = 0;
            }
        }
        if (g.pos() > end_bit) { fail(DS_EOF); break; }
        const int esc_code = (1 << pbits) - 1;
        /* FIXED subframes (the encoder's usual choice) predict from the last four samples held
         * in registers, not from the LDS ring; LPC subframes read the ring */
        const bool fx = t >= 8 && t <= 12;
        const int32_t fc0 = fx ? fixed_coef(order, 0) : 0, fc1 = fx ? fixed_coef(order, 1) : 0,
                      fc2 = fx ? fixed_coef(order, 2) : 0, fc3 = fx ? fixed_coef(order, 3) : 0;
        int32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0; /* samples i-1 .. i-4 */
        int rem = plen - order, param = 0, escw = -1;
        bool first = true, eof = false;
        int32_t* orow = a.out ? a.out + u * a.out_stride : nullptr;
        for (int i = 0; i < bs; ++i) {
            int64_t s;
            if (t == 0) {
                s = cval;
            } else if (t == 1) {
                s = g.sint(w);
            } else if (i < order) {
                s = ring[i][lane];
            } else {
                if (first || rem == 0) { /* get_rice_partition (decoder.py:400-411) */
                    if (!first) rem = plen;
                    first = false;
                    param = g.uint(pbits);
                    escw = -1;
                    if (param == esc_code) {
                        escw = g.uint(5);
                        if (escw == 0) { pfail(DS_ESC_ZERO); break; }
                    }
                }
                --rem;
                const int64_t r = escw >= 0 ? g.sint(escw) : g.rice(param, end_bit, eof);
                if (eof) { fail(DS_EOF); break; }
                int64_t acc = 0;
                if (fx) {
                    acc = (int64_t)fc0 * h0 + (int64_t)fc1 * h1 + (int64_t)fc2 * h2 + (int64_t)fc3 * h3;
                } else {
                    for (int j = 0; j < order; ++j) acc += (int64_t)coef[j][lane] * ring[(i - 1 - j) & 31][lane];
                }
                s = r + (acc >> shift);
            }
            ring[i & 31][lane] = (int32_t)s;
            h3 = h2;
            h2 = h1;
            h1 = h0;
            h0 = (int32_t)s;
            if ((i & 31) == 31 || i == bs - 1) { /* flush the ring column */
                const int c0 = i & ~31, cnt = i - c0 + 1;
                if (orow) {
                    if (cnt == 32) {
#pragma unroll
                        for (int k = 0; k < 32; k += 4) {
                            int4v v = {ring[k][lane], ring[k + 1][lane], ring[k + 2][lane], ring[k + 3][lane]};
                            *reinterpret_cast<int4v*>(orow + c0 + k) = v;
                        }
                    } else {
                        for (int k = 0; k < cnt; ++k) orow[c0 + k] = ring[k][lane];
                    }
                }
                if (cmp) {
                    if (cnt == 32 && a.expect_vec) { /* 16-byte loads of the source row */
                        if (a.expect_bytes == 2) {
                            const uint4* e4 = reinterpret_cast<const uint4*>((const int16_t*)a.expect + u * a.expect_stride + c0);
#pragma unroll
                            for (int g2 = 0; g2 < 4; ++g2) {
                                const uint4 v = e4[g2];
                                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                                for (int h = 0; h < 4; ++h) {
                                    bad += ring[8 * g2 + 2 * h][lane] != ((int32_t)(w[h] << 16) >> 16);
                                    bad += ring[8 * g2 + 2 * h + 1][lane] != ((int32_t)w[h] >> 16);
                                }
                            }
                        } else {
                            const int4v* e4 = reinterpret_cast<const int4v*>((const int32_t*)a.expect + u * a.expect_stride + c0);
#pragma unroll
                            for (int g2 = 0; g2 < 8; ++g2) {
                                const int4v v = e4[g2];
#pragma unroll
                                for (int h = 0; h < 4; ++h) bad += ring[4 * g2 + h][lane] != v[h];
                            }
                        }
                    } else {
                        for (int k = 0; k < cnt; ++k) bad += ring[k][lane] != expect_at(a, u, c0 + k);
                    }
                }
            }
            if (g.pos() > end_bit) { fail(DS_EOF); break; }
        }
        if (is_ref_error(st)) break;
    }
    if (!is_ref_error(st) && nch > 0) {
        /* footer (decoder.py:124-128): zero padding to a byte, CRC-16 */
        if (g.pos() & 7) {
            if (g.uint(8 - (int)(g.pos() & 7)) != 0) pfail(DS_PADDING);
        }
        const uint32_t crc16 = g.uint(16);
        if (g.pos() > end_bit) fail(DS_EOF);
        else {
            if ((g.pos() >> 3) != Fend) fail(DS_FRAME_END);
            if (a.check_crc) {
                uint32_t c;
                if ((g.pos() >> 3) == Fend && E > F) { /* the fused CRC: dwords not yet folded, then the tail */
                    c = g.crc;
                    const int64_t d0 = g.cnext, d1 = g.cend;
                    if (d1 > d0) c = crc16_more(a, crct, c, 4 * d0, 4 * d1);
                    if (4 * d1 >= Fh) c = crc16_more(a, crct, c, 4 * d1 > Fh ? 4 * d1 : Fh, E);
                } else {
                    c = crc16_range(a, crct, F, (g.pos() >> 3) - 2);
                }
                if (c != crc16) fail(DS_CRC16);
            }
        }
    }
    if (!is_ref_error(st) && neg_shift) fail(DS_NEG_SHIFT);
    if (bad) fail(DS_SAMPLES);
    a.status[f] = st;
    a.mismatch[f] = bad;
    a.decorr[f] = (decorr && !is_ref_error(st)) ? ((bs << 8) | ch_code) : 0;
}

/* The frames k_decode_fx listed (a.defer_all: every frame), one lane each. */
__global__ __launch_bounds__(kDecThreads) void k_decode(DecodeArgs a) {
    __shared__ int32_t ring[kRingSlots][kDecThreads];
    __shared__ int16_t coef[kRingSlots][kDecThreads]; /* precision <= 15 bits (4-bit field, 15 rejected) */
    __shared__ uint16_t crct[4 * 256];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4 * 256; i += kDecThreads) crct[i] = a.crc_slice[i];
    __syncthreads();
    const int64_t nl = a.defer_all ? a.n_frames : (int64_t)*a.defer_count;
    for (int64_t k = (int64_t)blockIdx.x * kDecThreads + lane; k < nl; k += (int64_t)gridDim.x * kDecThreads)
        decode_general(a, a.defer_all ? k : a.defer_list[k], ring, coef, crct, lane);
}

constexpr int kFxThreads = 256; /* k_decode_fx: frames per workgroup (one CRC table copy) */
constexpr int kFxGroup = 4;     /* CONSTANT / VERBATIM samples between comparisons (ring slots) */
constexpr int kFxRing = 16;     /* stream dwords a lane keeps in LDS ahead of its bit window */
constexpr int kFxLpc = 12;      /* the second pass's largest LPC order (history in registers) */
constexpr int kFxLpcW = 32;     /* ... for samples wider than 16 bits (that pass: no speculative blocks) */

/* k_decode_fx's reader.  Lanes read 64 unrelated frames, so a per-lane dword load that is
 * waited for at once would stall the whole wave about every sample.  Instead the window's
 * next dwords come from a per-lane LDS ring that the sample loop refills with one 16-byte
 * load per lane every 4 samples, at points common to all lanes, and lands 8 samples later.
 * A lane that outruns its ring (long codes, headers) reads the stream directly.
 * The window (hi, lo) is dwords k, k + 1 counted from the frame's first whole dword
 * cw = ceil(F / 4) (k starts at -1 for every frame alignment), nx is dword k + 2 (read one
 * dword ahead, so the ring's LDS latency is off the decode chain); the read position is
 * 32 (cw + k) + 32 - sh.  Ring slot j & 15 holds dword j for j in [k + 3, fe).  Dwords
 * k in [0, nfold) are folded into the CRC-16 as they leave the window (decode_general's
 * cnext / cend, relative; a separate wave-per-frame CRC pass measured slower). */
struct FxReader {
    const uint32_t* wb; /* dword cw */
    int32_t nrel;       /* wb[0 .. nrel) lie inside the stream */
    uint32_t hi, lo, nx;
    int32_t sh, k, knear, fe, fi; /* k >= knear: a 32-bit read could pass the stream's end;
                                     [fe, fi): dwords whose loads are in flight */
    uint32_t* sr;                 /* this lane's ring column: slot j at sr[j * kFxThreads] */
    uint32_t crc;                 /* CRC-16 of the frame's dwords k' in [0, min(k, nfold)) so far */
    int32_t nfold;
    const uint16_t* ct;
    __device__ __forceinline__ uint32_t direct(int32_t j) const {
        return (uint32_t)j < (uint32_t)nrel ? __builtin_bswap32(wb[j]) : 0u;
    }
    __device__ __forceinline__ uint32_t folded(uint32_t be) const { /* crc after one more whole dword */
        const uint32_t v = be ^ (crc << 16);
        return (uint32_t)ct[3 * 256 + (v >> 24)] ^ (uint32_t)ct[2 * 256 + ((v >> 16) & 0xFF)] ^
               (uint32_t)ct[256 + ((v >> 8) & 0xFF)] ^ (uint32_t)ct[v & 0xFF];
    }
    __device__ __forceinline__ void adv() {
        if ((uint32_t)k < (uint32_t)nfold) crc = folded(hi);
        hi = lo;
        lo = nx;
        ++k;
        const int32_t j = k + 2;
        nx = j < fe ? sr[(j & (kFxRing - 1)) * kFxThreads] : direct(j);
    }
    /* bits read since the frame's first whole dword, minus 32 */
    __device__ __forceinline__ int64_t rel() const { return 32 * (int64_t)k + 32 - sh; }
    __device__ __forceinline__ uint32_t peek32() const { return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh); }
    __device__ __forceinline__ void skip(int n) { /* 0 <= n <= 32 */
        sh -= n;
        if (sh < 0) {
            sh += 32;
            adv();
        }
    }
    __device__ __forceinline__ uint32_t uint(int n) {
        if (n == 0) return 0;
        const uint32_t v = peek32() >> (32 - n);
        skip(n);
        return v;
    }
    __device__ __forceinline__ uint64_t uint64(int n) {
        if (n <= 32) return uint(n);
        const uint64_t h = uint(n - 32);
        return (h << 32) | uint(32);
    }
    __device__ __forceinline__ int64_t sint(int n) {
        const uint64_t x = uint64(n);
        return n >= 64 ? (int64_t)x : (int64_t)(x << (64 - n)) >> (64 - n);
    }
    /* BitReader::rice with the end given relative (rel() > rend: past the stream's end) */
    __device__ __forceinline__ int64_t rice(int p2, int64_t rend, bool& eof) {
        uint64_t q = 0;
        uint32_t W = peek32();
        while (W == 0) {
            q += 32;
            skip(32);
            if (rel() > rend) {
                eof = true;
                return 0;
            }
            W = peek32();
        }
        const int z = __builtin_clz(W);
        q += z;
        uint64_t v;
        if (z + 1 + p2 <= 32) {
            v = (q << p2) | (p2 ? ((W << (z + 1)) >> (32 - p2)) : 0u);
            skip(z + 1 + p2);
        } else {
            skip(z + 1);
            v = (q << p2) | uint(p2);
        }
        return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
    }
    /* The refill pipeline.  Loads are started and landed unconditionally, a fixed number per
     * block, so the compiler's wait counts are exact (a load it cannot place in the count
     * makes it wait for every load in flight): a load that is not needed reads the CRC table
     * and lands in the trash slot kFxRing. */
    __device__ __forceinline__ void commit(const uint4& q, const bool valid) {
        auto slot = [&](int t) { return valid ? (fe + t) & (kFxRing - 1) : kFxRing; }; /* kFxRing: trash */
        sr[slot(0) * kFxThreads] = __builtin_bswap32(q.x);
        sr[slot(1) * kFxThreads] = __builtin_bswap32(q.y);
        sr[slot(2) * kFxThreads] = __builtin_bswap32(q.z);
        sr[slot(3) * kFxThreads] = __builtin_bswap32(q.w);
        fe += valid ? 4 : 0;
    }
    /* a lane that read past everything loaded or in flight restarts the ring after nx (the
     * caller drops its loads in flight) */
    __device__ __forceinline__ bool overtaken() {
        if (k + 3 <= fi) return false;
        fe = fi = k + 3;
        return true;
    }
    /* start the load of dwords [fi, fi + 4) when they fit the ring and the stream (true), else
     * of 16 harmless bytes at `dummy` (false) */
    __device__ __forceinline__ bool issue(uint4& q, const void* dummy) {
        const bool ok = fi + 4 - (k + 3) <= kFxRing && fi + 4 <= nrel;
        typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4))); /* dwords: 4-byte aligned */
        const u32x4a4 t = *reinterpret_cast<const u32x4a4*>(ok ? (const void*)(wb + fi) : dummy);
        q = uint4{t.x, t.y, t.z, t.w};
        fi += ok ? 4 : 0;
        return ok;
    }
};

/* the subframe's last cnt < 8 samples (ring slots [0, cnt)), after its sample loop */
template <int EB, bool OUT>
__device__ __forceinline__ bool fx_part(int32_t (*ring)[kFxThreads], const int lane, const void* erow, int32_t* orow,
                                        const int c0, const int cnt) {
    uint32_t bad = 0;
    for (int k = 0; k < cnt; ++k) {
        const int32_t x = ring[k][lane];
        if constexpr (OUT) orow[c0 + k] = x;
        if constexpr (EB == 2) bad |= (uint32_t)(x ^ (int32_t)((const int16_t*)erow)[c0 + k]);
        if constexpr (EB == 4) bad |= (uint32_t)(x ^ ((const int32_t*)erow)[c0 + k]);
    }
    return bad != 0;
}

/* k_decode_fx's frame: true when the frame decoded with every check passing and every sample
 * equal to the source row (status 0, mismatch 0); false hands it to k_decode, which decodes
 * it again from its first byte.  The checks are decode_general's, in its order, so a frame
 * this function accepts is one decode_general gives status 0 (it never reports a failure
 * itself). */
template <int EB, bool OUT, int LN>
__device__ __forceinline__ bool decode_fx(const DecodeArgs& a, const int64_t f, int32_t (*ring)[kFxThreads],
                                          int32_t (*wr)[kFxThreads], int32_t (*xr)[kFxThreads], uint32_t* sring,
                                          const uint16_t* crct, const int lane, bool& to_lpc) {
    FxReader g;
    int bs, nch, ss;
    /* the stream's last bit, relative as rel() (derived from wb: not kept in registers) */
    auto rend = [&]() __attribute__((always_inline)) { return a.stream_bytes * 8 - 32 * (int64_t)(g.wb - a.words); };
    {
        const int64_t F = a.offsets[f], Fend = a.offsets[f + 1];
        const int64_t cw = (F + 3) >> 2, E = Fend - 2;
        const int32_t fo = (int32_t)(32 * cw - 8 * F); /* frame-relative bit position = rel() + fo */
        g.wb = a.words + cw;
        const int64_t nr = a.n_words - cw;
        g.nrel = nr < 0 ? 0 : nr > 0x7fffffff ? 0x7fffffff : (int32_t)nr;
        g.hi = (cw - 1 >= 0 && cw - 1 < a.n_words) ? __builtin_bswap32(a.words[cw - 1]) : 0u;
        g.lo = g.direct(0);
        g.nx = g.direct(1);
        g.sh = fo;
        g.k = -1;
        g.fe = g.fi = 2;
        g.sr = sring + lane;
        g.ct = crct;
        g.crc = 0;
        g.nfold = 0;
        if (a.check_crc && E > F) {
            const int64_t nf = (E >> 2) - cw;
            g.nfold = nf < 0 ? 0 : nf > 0x7fffffff ? 0x7fffffff : (int32_t)nf;
            g.crc = crc16_more(a, crct, 0u, F, E < 4 * cw ? E : 4 * cw);
        }
        const int64_t kn = ((a.stream_bytes * 8) >> 5) - 1 - cw;
        g.knear = kn < -1 ? -1 : kn > 0x7fffffff ? 0x7fffffff : (int32_t)kn;

        /* ---- frame header (decoder.py:133-245) ---- */
        if (g.uint(15) != 0x7FFC) return false;
        (void)g.uint(1);
        const int bcode = g.uint(4);
        if (!(bcode > 0 && bcode < 15)) return false;
        const int rcode = g.uint(4);
        if (rcode == 15) return false;
        const int ch_code = g.uint(4);
        if (ch_code > 7) return false; /* stereo decorrelation (8..10) and reserved codes: k_decode */
        const int scode = g.uint(3);
        if (scode == 3) return false;
        if (g.uint(1) != 0) return false;
        const uint32_t b0 = g.uint(8);
        const int extra = b0 >= 0xFE ? 6 : b0 >= 0xFC ? 5 : b0 >= 0xF8 ? 4 : b0 >= 0xF0 ? 3 : b0 >= 0xE0 ? 2 : b0 >= 0xC0 ? 1 : 0;
        uint64_t fno = extra == 0 ? b0 : (b0 & ((1u << (6 - extra)) - 1));
        for (int k = 0; k < extra; ++k) fno = (fno << 6) | (g.uint(8) & 0x3F);
        if (bcode == 1) bs = 192;
        else if (bcode <= 5) bs = 144 << bcode;
        else if (bcode == 6) bs = (int)g.uint(8) + 1;
        else if (bcode == 7) bs = (int)g.uint(16) + 1;
        else bs = 1 << bcode;
        if (rcode == 12) (void)g.uint(8);
        else if (rcode == 13 || rcode == 14) (void)g.uint(16);
        const int hdr_bytes = (int)((g.rel() + fo) >> 3);
        const uint32_t crc8 = g.uint(8);
        if (g.rel() > rend()) return false;
        if (a.check_crc) {
            const uint8_t* bytes = reinterpret_cast<const uint8_t*>(a.words);
            uint32_t c = 0;
            for (int k = 0; k < hdr_bytes; ++k) {
                c ^= bytes[F + k];
                for (int bt = 0; bt < 8; ++bt) c = (c & 0x80) ? ((c << 1) ^ 0x07) & 0xFF : (c << 1) & 0xFF;
            }
            if (c != crc8) return false;
        }
        ss = scode == 0 ? a.sample_size : sample_size_of(scode);
        nch = ch_code == 1 ? a.channels : ch_code + 1;
        if (nch != a.channels) return false;
        if (a.first_frame >= 0 && (int64_t)fno != a.first_frame + f) return false;
        if (OUT && bs > a.out_stride) return false;
    }

    /* ---- subframes: CONSTANT, VERBATIM, FIXED (decoder.py:267-421, 473-498) ---- */
    for (int c = 0; c < nch; ++c) {
        const int64_t u = f * a.channels + c;
        if (EB && unit_len_d(a, u) != bs) return false;
        const void* erow = EB == 2 ? (const void*)((const int16_t*)a.expect + u * a.expect_stride)
                                   : (const void*)((const int32_t*)a.expect + u * a.expect_stride);
        int32_t* orow = OUT ? a.out + u * a.out_stride : nullptr;
        if (g.uint(1) != 0) return false;
        const int t = g.uint(6);
        /* LPC (LN > 0: orders up to LN) and invalid types: k_decode */
        if (!(t <= 1 || (t >= 8 && t <= 12) || (LN > 0 && t >= 32 && (t & 31) < LN))) {
            /* worth the LPC pass: measured on 16-bit streams (config 2 open mixes 36.6 -> 25.4 ms);
             * on config 3's open mix (24-bit stereo, L 32) it cost 103 -> 116 ms, so wider
             * samples go straight to k_decode */
            to_lpc = LN == 0 && t >= 32 && (t & 31) < (a.sample_size <= 16 ? kFxLpc : kFxLpcW);
            return false;
        }
        if (g.uint(1)) return false;                        /* wasted bits: k_decode */
        const int w = ss;
        if (t <= 1) {
            const int64_t cval = t == 0 ? g.sint(w) : 0;
            for (int i = 0; i < bs; ++i) {
                ring[i & (kFxGroup - 1)][lane] = (int32_t)(t == 0 ? cval : g.sint(w));
                if ((i & (kFxGroup - 1)) == kFxGroup - 1 || i == bs - 1)
                    if (fx_part<EB, OUT>(ring, lane, erow, orow, i & ~(kFxGroup - 1), (i & (kFxGroup - 1)) + 1)) return false;
                if (g.rel() > rend()) return false;
            }
            continue;
        }
        /* FIXED: the warm-up samples, then x[i] = r + the order-k prediction, restored as k
         * running differences: with d_j = Delta^j x[i-1], Delta^k x[i] = r and Delta^j x[i] =
         * Delta^(j+1) x[i] + d_j.  Wrapping 32-bit arithmetic gives the reference's value
         * modulo 2^32, which is what the int32 ring keeps (decode_general: int32 history). */
        /* LPC (LN > 0, order <= LN): the last LN samples h[0] = x[i-1] .. and the quantised
         * coefficients in registers (static indices: every loop over them is unrolled to LN);
         * x[i] = r + (sum c_j h_j >> shift), the sum in int64 over the int32 history as
         * decode_general's ring (decoder.py:490-498) */
        const bool lpc = LN > 0 && t >= 32;
        const int order = lpc ? (t & 31) + 1 : t & 7;
        uint32_t h[LN > 0 ? LN : 1];
        int32_t cf[LN > 0 ? LN : 1];
        int shift = 0;
#pragma unroll
        for (int j = 0; j < (LN > 0 ? LN : 1); ++j) h[j] = 0, cf[j] = 0;
        uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
        uint32_t wbad = 0; /* the warm-up samples are compared (and written) as they are read */
        for (int k = 0; k < order; ++k) {
            const uint32_t x = (uint32_t)g.sint(w);
            if constexpr (OUT) orow[k] = (int32_t)x;
            if constexpr (EB == 2) wbad |= x ^ (uint32_t)(int32_t)((const int16_t*)erow)[k];
            if constexpr (EB == 4) wbad |= x ^ (uint32_t)((const int32_t*)erow)[k];
            const uint32_t u1 = x - d0, u2 = u1 - d1, u3 = u2 - d2;
            d0 = x;
            d1 = u1;
            d2 = u2;
            d3 = u3;
            if constexpr (LN > 0) {
#pragma unroll
                for (int j = LN - 1; j > 0; --j) h[j] = h[j - 1];
                h[0] = x;
            }
        }
        if constexpr (LN > 0) {
            if (lpc) { /* decoder.py:286-300: precision, shift, coefficients */
                const int prec = g.uint(4);
                if (prec == 15) return false;
                shift = (int)g.sint(5);
                if (shift < 0) return false; /* decode_general reports it after the frame */
#pragma unroll
                for (int j = 0; j < LN; ++j) cf[j] = j < order ? (int32_t)g.sint(prec + 1) : 0;
                d0 = d1 = d2 = d3 = 0;
            }
        }
        /* the levels the order uses, as lane masks (v_cndmask on SGPR pairs, no VGPRs) */
        const bool m0 = !lpc && order > 0, m1 = !lpc && order > 1, m2 = !lpc && order > 2, m3 = !lpc && order > 3;
        d0 = m0 ? d0 : 0u;
        d1 = m1 ? d1 : 0u;
        d2 = m2 ? d2 : 0u;
        d3 = m3 ? d3 : 0u;
        const int cm = g.uint(2);
        if (cm > 1) return false;
        const int pbits = cm ? 5 : 4;
        const int po = g.uint(4);
        if ((bs & ((1 << po) - 1)) != 0 || (bs >> po) <= order) return false;
        const int plen = bs >> po;
        if (g.rel() > rend()) return false;
        int rem = 0, next = plen - order, param = 0;
        bool esc = false;
        /* the sample loop runs in blocks of 4 samples common to the lanes of the wave.  Two
         * loads of each kind are in flight per lane, in register slots alternating by block:
         * at block B the slot B & 1 commits the stream's oldest 16 bytes into the LDS ring and
         * this block's 4 source-row samples into the lane's LDS slots (both loaded at block
         * B - 2), then starts the next stream load and block B + 2's source-row load. */
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        typedef typename std::conditional<EB == 4, u32x4, u32x2>::type ExpV;
        /* the source row's block at sample i when it lies inside the row, else the CRC table */
        const void* dummy = a.crc_slice;
        auto exp_load = [&](int i) __attribute__((always_inline)) -> ExpV {
            const bool in = i + 4 <= bs;
            const void* p2 = !in ? dummy : EB == 4 ? (const void*)((const int32_t*)erow + i) : (const void*)((const int16_t*)erow + i);
            return *reinterpret_cast<const ExpV*>(p2);
        };
        /* the prologue starts the loads in the loop's own order (stream, row, stream, row), so
         * the wait counts on entering the loop match those around its back edge */
        ExpV qe0{}, qe1{};
        uint4 q0, q1;
        g.overtaken();
        bool si0 = g.issue(q0, dummy);
        if constexpr (EB != 0) qe0 = exp_load(0);
        bool si1 = g.issue(q1, dummy);
        if constexpr (EB != 0) qe1 = exp_load(4);
        uint32_t bad = wbad;
        bool fail = false;
        auto expect_commit = [&](const ExpV& qe) __attribute__((always_inline)) {
            int32_t e[4];
            if constexpr (EB == 4) {
                e[0] = (int32_t)qe[0], e[1] = (int32_t)qe[1], e[2] = (int32_t)qe[2], e[3] = (int32_t)qe[3];
            } else {
                e[0] = (int32_t)(qe[0] << 16) >> 16, e[1] = (int32_t)qe[0] >> 16;
                e[2] = (int32_t)(qe[1] << 16) >> 16, e[3] = (int32_t)qe[1] >> 16;
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) xr[kk][lane] = e[kk];
        };
        /* x[i] from its residual: FIXED by the running differences, LPC by the history */
        auto restore = [&](const uint32_t r) __attribute__((always_inline)) -> uint32_t {
            if constexpr (LN > 0) {
                if (lpc) {
                    int64_t acc = 0;
#pragma unroll
                    for (int j = 0; j < LN; ++j) acc += (int64_t)cf[j] * (int64_t)(int32_t)h[j];
                    const uint32_t x = r + (uint32_t)(acc >> shift);
#pragma unroll
                    for (int j = LN - 1; j > 0; --j) h[j] = h[j - 1];
                    h[0] = x;
                    return x;
                }
            }
            const uint32_t u3 = r + d3, u2 = u3 + d2, u1 = u2 + d1, x = u1 + d0;
            d0 = m0 ? x : 0u;
            d1 = m1 ? u1 : 0u;
            d2 = m2 ? u2 : 0u;
            d3 = m3 ? u3 : 0u;
            return x;
        };
        /* samples [i0, i0 + 4) (those below bs).  MID: a block every lane has whole and past its
         * warm-up (i0 >= 4, i0 + 4 <= bs): no per-sample bounds, the source row from the LDS
         * slots, and a Rice code's window advance without a branch (its next dword read from
         * the ring, which the fast-path condition guarantees holds it). */
        auto sample = [&](const int i0, const int kk, auto mid_t) __attribute__((always_inline)) {
            constexpr bool MID = decltype(mid_t)::value;
            {
                const int i = i0 + kk;
                if (MID || (i < bs && i >= order)) { /* warm-up samples: compared as read */
                    uint32_t x;
                    {
                        const uint32_t W = g.peek32();
                        const int z = __builtin_clz(W | 1u);
                        const int nb = z + 1 + param;
                        uint32_t r;
                        if (W == 0 || nb > 32 || rem == 0 || esc || g.k >= g.knear || (MID && g.k + 3 >= g.fe)) {
                            if (rem == 0) { /* get_rice_partition (decoder.py:400-411) */
                                rem = next;
                                next = plen;
                                param = g.uint(pbits);
                                esc = param == (1 << pbits) - 1;
                                if (esc) {
                                    param = g.uint(5); /* the escaped partition's sample width */
                                    if (param == 0) fail = true;
                                }
                            }
                            bool eof = false;
                            r = (uint32_t)(esc ? g.sint(param) : g.rice(param, rend(), eof));
                            if (eof || g.rel() > rend()) fail = true;
                        } else {
                            /* the unary run (z zeros), the stop bit and param low bits lie in
                             * W: (W << z) >> (31 - param) = 2^param + low, so v = (z << param)
                             * + low; no read can pass the stream's end (k < knear) */
                            const uint32_t v = ((W << z) >> (31 - param)) + ((uint32_t)(z - 1) << param);
                            if constexpr (MID) {
                                const int32_t sh2 = g.sh - nb;
                                const bool c = sh2 < 0;
                                const uint32_t nn = g.sr[((g.k + 3) & (kFxRing - 1)) * kFxThreads];
                                const uint32_t fc = g.folded(g.hi);
                                g.crc = c && (uint32_t)g.k < (uint32_t)g.nfold ? fc : g.crc;
                                g.hi = c ? g.lo : g.hi;
                                g.lo = c ? g.nx : g.lo;
                                g.nx = c ? nn : g.nx;
                                g.k += c ? 1 : 0;
                                g.sh = c ? sh2 + 32 : sh2;
                            } else {
                                g.skip(nb);
                            }
                            r = (v >> 1) ^ (0u - (v & 1u));
                        }
                        --rem;
                        x = restore(r);
                    }
                    if constexpr (OUT) orow[i] = (int32_t)x;
                    if constexpr (EB != 0) {
                        /* a block that ends past bs has no committed slots: the row directly */
                        const int32_t e = MID || i0 + 4 <= bs ? xr[kk][lane]
                                                              : (EB == 2 ? (int32_t)((const int16_t*)erow)[i] : ((const int32_t*)erow)[i]);
                        bad |= x ^ (uint32_t)e;
                    }
                }
            }
        };
        /* A middle block whose 4 samples need no partition header, escape, stream-end or ring
         * check (tested once, at its start) decodes speculatively: each sample on the fast path,
         * its only per-sample hazard (a code longer than the 32-bit window) collected in a lane
         * flag.  If any lane raised it, the state saved at the block's start is restored and the
         * general sample path redoes the block. */
        auto mid_sample = [&](const int i0, const int kk, uint32_t& hz, uint32_t& bb) __attribute__((always_inline)) {
            const uint32_t W = g.peek32();
            const int z = __builtin_clz(W | 1u);
            const int nb = z + 1 + param;
            hz |= (uint32_t)(W == 0) | (uint32_t)(nb > 32);
            const uint32_t v = ((W << z) >> (31 - param)) + ((uint32_t)(z - 1) << param);
            const int32_t sh2 = g.sh - nb;
            const bool c = sh2 < 0; /* the window advances one dword (its next from the ring) */
            const uint32_t nn = g.sr[((g.k + 3) & (kFxRing - 1)) * kFxThreads];
            const uint32_t fc = g.folded(g.hi);
            g.crc = c && (uint32_t)g.k < (uint32_t)g.nfold ? fc : g.crc;
            g.hi = c ? g.lo : g.hi;
            g.lo = c ? g.nx : g.lo;
            g.nx = c ? nn : g.nx;
            g.k += c ? 1 : 0;
            g.sh = c ? sh2 + 32 : sh2;
            const uint32_t r = (v >> 1) ^ (0u - (v & 1u));
            const uint32_t x = restore(r);
            if constexpr (OUT) orow[i0 + kk] = (int32_t)x;
            if constexpr (EB != 0) bb |= x ^ (uint32_t)xr[kk][lane];
        };
        auto block = [&](const int i0) __attribute__((always_inline)) {
            const bool whole = i0 >= 4 && i0 + 4 <= bs;
            const bool calm = rem >= 4 && !esc && g.k + 3 < g.knear && g.k + 6 < g.fe;
            if (LN <= kFxLpc && __builtin_amdgcn_ballot_w64(!(whole && calm)) == 0) { /* wave-uniform */
                const uint32_t s_hi = g.hi, s_lo = g.lo, s_nx = g.nx, s_crc = g.crc;
                const int32_t s_sh = g.sh, s_k = g.k;
                const uint32_t s_d0 = d0, s_d1 = d1, s_d2 = d2, s_d3 = d3;
                uint32_t s_h[LN > 0 ? LN : 1];
                if constexpr (LN > 0) {
#pragma unroll
                    for (int j = 0; j < LN; ++j) s_h[j] = h[j];
                }
                uint32_t hz = 0, bb = 0;
                mid_sample(i0, 0, hz, bb);
                mid_sample(i0, 1, hz, bb);
                mid_sample(i0, 2, hz, bb);
                mid_sample(i0, 3, hz, bb);
                if (__builtin_amdgcn_ballot_w64(hz != 0) == 0) {
                    rem -= 4;
                    bad |= bb;
                    return;
                }
                g.hi = s_hi, g.lo = s_lo, g.nx = s_nx, g.crc = s_crc, g.sh = s_sh, g.k = s_k;
                d0 = s_d0, d1 = s_d1, d2 = s_d2, d3 = s_d3;
                if constexpr (LN > 0) {
#pragma unroll
                    for (int j = 0; j < LN; ++j) h[j] = s_h[j];
                }
            }
#pragma unroll 1
            for (int kk = 0; kk < 4; ++kk) sample(i0, kk, std::false_type{});
        };
        /* two blocks per iteration, each with its own register slot (no copies of registers
         * whose loads are in flight: a copy would wait for them) */
        for (int i0 = 0; i0 < bs; i0 += 8) {
            g.commit(q0, si0);
            if constexpr (EB != 0) expect_commit(qe0);
            if (g.overtaken()) si1 = false;
            si0 = g.issue(q0, dummy);
            if constexpr (EB != 0) qe0 = exp_load(i0 + 8);
            block(i0);
            if (fail || bad) break; /* a failed check (escape width 0, end of stream) or a difference */
            g.commit(q1, si1);
            if constexpr (EB != 0) expect_commit(qe1);
            if (g.overtaken()) si0 = false;
            si1 = g.issue(q1, dummy);
            if constexpr (EB != 0) qe1 = exp_load(i0 + 12);
            block(i0 + 4);
            if (fail || bad) break;
        }
        if (fail || bad) return false;
        /* the stream loads still in flight, oldest first */
        g.commit(q0, si0);
        g.commit(q1, si1);
    }
    /* ---- footer (decoder.py:124-128) ---- */
    if (g.rel() & 7) {
        if (g.uint(8 - (int)(g.rel() & 7)) != 0) return false;
    }
    const uint32_t crc16 = g.uint(16);
    if (g.rel() > rend()) return false;
    /* re-read (volatile: not kept live in registers through the sample loops) */
    const int64_t F = *(volatile const int64_t*)(a.offsets + f), Fend = *(volatile const int64_t*)(a.offsets + f + 1);
    const int64_t cw = (F + 3) >> 2, E = Fend - 2;
    if (((g.rel() + 32 * cw - 8 * F) >> 3) != Fend - F) return false;
    if (a.check_crc) {
        uint32_t c = g.crc;
        if (E > F) {
            /* dwords [cw + min(max(k, 0), nfold), cw + nfold) have not left the window yet */
            const int32_t done = g.k < 0 ? 0 : g.k < g.nfold ? g.k : g.nfold;
            if (g.nfold > done) c = crc16_more(a, crct, c, 4 * (cw + done), 4 * (cw + g.nfold));
            if ((E >> 2) >= cw) c = crc16_more(a, crct, c, 4 * (E >> 2) > 4 * cw ? 4 * (E >> 2) : 4 * cw, E);
        } else {
            c = crc16_range(a, crct, F, E);
        }
        if (c != crc16) return false;
    }
    return true;
}

/* LN = 0: every frame; LN > 0: the frames the LN = 0 pass listed (defer_list), FIXED and LPC
 * subframes of order <= LN, listing what it cannot vouch for in defer2_list */
template <int EB, bool OUT, int LN>
__global__ __launch_bounds__(kFxThreads) __attribute__((amdgpu_waves_per_eu(EB == 0 && !OUT ? 8 : 7, 8))) void k_decode_fx(DecodeArgs a) {
    /* per-lane columns: a CONSTANT / VERBATIM subframe's samples between flushes, or a FIXED
     * subframe's source-row block of 4; a lane is in one kind of subframe at a time */
    __shared__ int32_t ring[kFxGroup][kFxThreads];
    __shared__ uint32_t sring[(kFxRing + 1) * kFxThreads]; /* + the trash slot */
    __shared__ uint16_t crct[4 * 256];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4 * 256; i += kFxThreads) crct[i] = a.crc_slice[i];
    __syncthreads();
    const int64_t kf = (int64_t)blockIdx.x * kFxThreads + lane;
    if (kf >= (LN > 0 ? (int64_t)*a.defer_count : a.n_frames)) return;
    const int64_t f = LN > 0 ? a.defer_list[kf] : kf;
    bool to_lpc = false;
    if (decode_fx<EB, OUT, LN>(a, f, ring, ring, ring, sring, crct, lane, to_lpc)) {
        a.status[f] = 0;
        a.mismatch[f] = 0;
        a.decorr[f] = 0;
    } else {
        /* the first pass lists a frame for the LPC pass only when an LPC subframe of order <= kFxLpc
         * stopped it; anything else goes straight to k_decode's list */
        const bool l1 = LN == 0 && to_lpc && a.lpc_pass;
        const unsigned long long k = atomicAdd(l1 ? a.defer_count : a.defer2_count, 1ull);
        (l1 ? a.defer_list : a.defer2_list)[k] = f;
    }
}

/* Interchannel decorrelation (decoder.py:431-448) of the frames k_decode marked, in place,
 * then the comparison with the source rows. */
__global__ __launch_bounds__(256) void k_decorr(DecodeArgs a) {
    const int64_t f = blockIdx.x;
    const int32_t d = a.decorr[f];
    if (d == 0) return;
    const int code = d & 0xFF, bs = d >> 8;
    int32_t* r0 = a.out + (f * a.channels) * a.out_stride;
    int32_t* r1 = r0 + a.out_stride;
    int64_t bad = 0;
    for (int i = threadIdx.x; i < bs; i += blockDim.x) {
        const int32_t s0 = r0[i], s1 = r1[i];
        int32_t l, r;
        if (code == 8) { l = s0; r = s0 - s1; }             /* L_S */
        else if (code == 9) { l = s0 + s1; r = s1; }        /* S_R */
        else { r = s0 - (s1 >> 1); l = r + s1; }            /* M_S */
        r0[i] = l;
        r1[i] = r;
        if (a.expect && unit_len_d(a, f * a.channels) == bs && unit_len_d(a, f * a.channels + 1) == bs)
            bad += (l != expect_at(a, f * a.channels, i)) + (r != expect_at(a, f * a.channels + 1, i));
    }
    __shared__ unsigned long long tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    if (bad) atomicAdd(&tot, (unsigned long long)bad);
    __syncthreads();
    if (threadIdx.x == 0 && tot) {
        a.mismatch[f] += (int64_t)tot;
        if (a.status[f] == 0) a.status[f] = dstat(DS_SAMPLES);
    }
}

hipError_t launch_decode(DecodeArgs a, hipStream_t s) {
    if (a.n_frames <= 0) return hipSuccess;
    int64_t blocks = (a.n_frames + kDecThreads - 1) / kDecThreads;
    if (!a.defer_all && !(a.expect && !a.expect_vec) && !(a.out && (a.out_stride & 3))) {
        hipError_t e = hipMemsetAsync(a.defer_count, 0, sizeof(unsigned long long), s);
        if (e != hipSuccess) return e;

        const dim3 g((unsigned)((a.n_frames + kFxThreads - 1) / kFxThreads)), b(kFxThreads);
        const int eb = a.expect ? a.expect_bytes : 0;
        auto fx = [&](auto ln) {
            constexpr int LN = decltype(ln)::value;
            if (a.out) {
                if (eb == 2) hipLaunchKernelGGL((k_decode_fx<2, true, LN>), g, b, 0, s, a);
                else if (eb == 4) hipLaunchKernelGGL((k_decode_fx<4, true, LN>), g, b, 0, s, a);
                else hipLaunchKernelGGL((k_decode_fx<0, true, LN>), g, b, 0, s, a);
            } else {
                if (eb == 2) hipLaunchKernelGGL((k_decode_fx<2, false, LN>), g, b, 0, s, a);
                else if (eb == 4) hipLaunchKernelGGL((k_decode_fx<4, false, LN>), g, b, 0, s, a);
                else hipLaunchKernelGGL((k_decode_fx<0, false, LN>), g, b, 0, s, a);
            }
            return hipGetLastError();
        };
        /* the listed frames again, with LPC subframes of order <= kFxLpc; the rest for k_decode */
        static const bool lpc_pass = [] {
            const char* v = getenv("FLACMI_DECODE_LPC");
            return !(v && v[0] == '0');
        }();
        a.lpc_pass = lpc_pass;
        if ((e = hipMemsetAsync(a.defer2_count, 0, sizeof(unsigned long long), s)) != hipSuccess) return e;
        if ((e = fx(std::integral_constant<int, 0>{})) != hipSuccess) return e;
        if (lpc_pass) {
            e = a.sample_size <= 16 ? fx(std::integral_constant<int, kFxLpc>{}) : fx(std::integral_constant<int, kFxLpcW>{});
            if (e != hipSuccess) return e;
        }
        a.defer_count = a.defer2_count;
        a.defer_list = a.defer2_list;
        blocks = blocks < 2048 ? blocks : 2048; /* the listed frames: a grid-stride loop */
    } else {
        a.defer_all = 1; /* rows k_decode_fx cannot read with 16-byte accesses: every frame general */
    }
    hipLaunchKernelGGL(k_decode, dim3((unsigned)blocks), dim3(kDecThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !a.out) return e;
    hipLaunchKernelGGL(k_decorr, dim3((unsigned)a.n_frames), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace flacmi
