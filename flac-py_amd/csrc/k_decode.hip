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
 *   k_decode   one LANE per frame.  Each lane walks its frame with a 64-bit big-endian
 *              bit window refilled one dword at a time (frames start at any byte) and
 *              decodes a Rice code with one v_ffbh.  Sample i of every lane's subframe is
 *              restored in loop iteration i, so the lanes of a wave stay in lock-step and
 *              the per-lane history ring in LDS (32 slots x 64 lanes, slot-major: a lane's
 *              column is one bank) is conflict-free.  Every 32 samples a lane flushes its
 *              ring column as 128 contiguous bytes of its decoded row and compares them with
 *              the source row.  CRC-8 / CRC-16 are recomputed from the frame bytes with the
 *              writer's slice-by-4 table (the reference reads them unchecked).
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

/* MSB-first reader over the stream: `buf` holds the 64 bits that start at dword `bw`. */
struct BitReader {
    const uint32_t* w;
    int64_t nw;
    int64_t pos; /* absolute bit position */
    int64_t bw;
    uint64_t buf;
    /* CRC-16 of the frame folded as whole dwords leave the window, in stream order: dword
     * cnext is the next one due, dwords below cend are inside the CRC range (crc16_fused) */
    const uint16_t* ct = nullptr;
    uint32_t crc = 0;
    int64_t cnext = 0, cend = 0;
    __device__ __forceinline__ uint32_t ld(int64_t i) const { return i < nw ? __builtin_bswap32(w[i]) : 0u; }
    __device__ __forceinline__ void fold(uint32_t be) { /* one whole big-endian dword */
        const uint32_t v = be ^ (crc << 16);
        crc = ct[3 * 256 + (v >> 24)] ^ ct[2 * 256 + ((v >> 16) & 0xFF)] ^ ct[256 + ((v >> 8) & 0xFF)] ^ ct[v & 0xFF];
    }
    __device__ __forceinline__ void seek(int64_t p) {
        pos = p;
        bw = p >> 5;
        buf = ((uint64_t)ld(bw) << 32) | ld(bw + 1);
    }
    /* the 32 bits at pos, MSB first */
    __device__ __forceinline__ uint32_t peek32() {
        int64_t off = pos - (bw << 5);
        if (off > 32) {
            if (off < 64) {
                if (ct && bw == cnext && bw < cend) { /* dword bw leaves the window */
                    fold((uint32_t)(buf >> 32));
                    ++cnext;
                }
                buf = (buf << 32) | ld(bw + 2);
                bw += 1;
                off -= 32;
            } else {
                seek(pos);
                off = pos & 31;
            }
        }
        return (uint32_t)((buf << off) >> 32);
    }
    __device__ __forceinline__ uint32_t uint(int n) { /* 0 <= n <= 32 (binary.py:97) */
        if (n == 0) return 0;
        const uint32_t v = peek32() >> (32 - n);
        pos += n;
        return v;
    }
    __device__ __forceinline__ uint64_t uint64(int n) { /* 0 <= n <= 64 */
        if (n <= 32) return uint(n);
        const uint64_t hi = uint(n - 32);
        return (hi << 32) | uint(32);
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
            pos += 32;
            if (pos > end) {
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
            pos += z + 1 + p;
        } else {
            pos += z + 1;
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

__global__ __launch_bounds__(kDecThreads) void k_decode(DecodeArgs a) {
    __shared__ int32_t ring[kRingSlots][kDecThreads];
    __shared__ int16_t coef[kRingSlots][kDecThreads]; /* precision <= 15 bits (4-bit field, 15 rejected) */
    __shared__ uint16_t crct[4 * 256];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4 * 256; i += kDecThreads) crct[i] = a.crc_slice[i];
    __syncthreads();

    const int64_t f = (int64_t)blockIdx.x * kDecThreads + lane;
    if (f >= a.n_frames) return;
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
    g.seek(F * 8);
    /* a parse failure after the reader ran off the stream is the EOFError of that read */
    auto pfail = [&](int32_t site) { fail(g.pos > end_bit ? (int32_t)DS_EOF : site); };

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
        const int hdr_bytes = (int)((g.pos >> 3) - F); /* byte-aligned here */
        const uint32_t crc8 = g.uint(8);
        if (g.pos > end_bit) { pfail(DS_EOF); break; }
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
                if (g.pos > end_bit) break;
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
        if (g.pos > end_bit) { fail(DS_EOF); break; }
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
            if (g.pos > end_bit) { fail(DS_EOF); break; }
        }
        if (is_ref_error(st)) break;
    }
    if (!is_ref_error(st) && nch > 0) {
        /* footer (decoder.py:124-128): zero padding to a byte, CRC-16 */
        if (g.pos & 7) {
            if (g.uint(8 - (int)(g.pos & 7)) != 0) pfail(DS_PADDING);
        }
        const uint32_t crc16 = g.uint(16);
        if (g.pos > end_bit) fail(DS_EOF);
        else {
            if ((g.pos >> 3) != Fend) fail(DS_FRAME_END);
            if (a.check_crc) {
                uint32_t c;
                if ((g.pos >> 3) == Fend && E > F) { /* the fused CRC: dwords not yet folded, then the tail */
                    c = g.crc;
                    const int64_t d0 = g.cnext, d1 = g.cend;
                    if (d1 > d0) c = crc16_more(a, crct, c, 4 * d0, 4 * d1);
                    if (4 * d1 >= Fh) c = crc16_more(a, crct, c, 4 * d1 > Fh ? 4 * d1 : Fh, E);
                } else {
                    c = crc16_range(a, crct, F, (g.pos >> 3) - 2);
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

hipError_t launch_decode(const DecodeArgs& a, hipStream_t s) {
    if (a.n_frames <= 0) return hipSuccess;
    const int64_t blocks = (a.n_frames + kDecThreads - 1) / kDecThreads;
    hipLaunchKernelGGL(k_decode, dim3((unsigned)blocks), dim3(kDecThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !a.out) return e;
    hipLaunchKernelGGL(k_decorr, dim3((unsigned)a.n_frames), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace flacmi
