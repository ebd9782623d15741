/* k_frame.hip — the FLAC frame writer on the device (residual bit
 * packing and frame assembly).
 *
 * The reference writes every frame on the host one bit at a time through binary.Put:
 *   frame header   encoder.py:194-234 (sync code, block-size / rate / channel / size codes,
 *                  coded_number.py:7-39 frame number, CRC-8 crc.py:18-22)
 *   subframes      encoder.py:553-627 (type byte, warm-up samples, LPC precision / shift /
 *                  coefficients), put_residual :765-806 (coding method, partition order,
 *                  per partition the parameter and the Rice codes: x >> p zeros, a one,
 *                  the low p bits)
 *   footer         encoder.py:159-163 (zero padding to a byte, CRC-16 crc.py:25-31)
 *
 * Here:
 *   k_frame_sizes  one wave per frame: exact frame size from the analysis metadata
 *                  (meta.rice_bits is the reference's size estimate, which counts 4 + 4|5
 *                  header bits per partition; the written size differs from it by a
 *                  closed form), the frame's status (first reference exception), then a
 *                  three-kernel exclusive scan gives every frame its byte offset.
 *   k_pack         one workgroup per frame.  Every field is OR-ed into an LDS window of
 *                  kWinWords 32-bit words at its exact bit position (positions from a
 *                  workgroup scan of per-value code lengths, 8 values per thread); a full
 *                  window is flushed to HBM with coalesced dword stores (byte stores only
 *                  on the frame's first and last word, which it shares with its
 *                  neighbours).  The CRC-16 is computed on the fly: each thread folds its
 *                  contiguous run of window words with slice-by-4 tables and moves the
 *                  partial CRC to the frame's end with x^(8d) tables (the CRC is linear
 *                  and starts from 0, so CRC(A||B) = CRC(A)*x^(8|B|) + CRC(B) mod P).
 *                  The general writer: 64-bit residuals, partitions under 8 values and
 *                  the frames the two kernels below hand over by list.
 *   k_packw        the default for 32-bit residual rows: one wave per frame, a 2 KB (samples
 *                  of <= 16 bits) or 4 KB LDS ring, finished 512-byte chunks leaving it as
 *                  the tiles advance.
 *   k_pack32       (knob FLACMI_PACK_GENERIC=2) frames that fit one LDS window (12 KB when
 *                  a verbatim frame fits it, else 16 KB): contiguous chunk runs per
 *                  thread, one scan per subframe.
 *
 * Bit coordinates inside k_pack are "aligned": bit 0 is the MSB of the 32-bit word that
 * holds the frame's first byte, so window word k is output word (F >> 2) + wb + k.  The
 * window words hold bits MSB first; stores byte-swap them. */
#include "device_common.h"

#include <cstdlib>

namespace flacmi {

constexpr int kWinWords = 4096;           /* 16 KB LDS window */
constexpr int kWinSmall = 3072;           /* k_pack32's window for frames of <= ~9.8 KB */
constexpr int kPackThreads = 256;
constexpr int kCrcPowLevels = 28;         /* frames < 2^28 bytes */

/* block-size code (encoder.py:245-255, common.py:85-105): 0 = not encodable */
__device__ __forceinline__ int bs_code(int bs) {
    switch (bs) {
        case 192: return 1;
        case 576: return 2;
        case 1152: return 3;
        case 2304: return 4;
        case 4608: return 5;
        case 256: return 8;
        case 512: return 9;
        case 1024: return 10;
        case 2048: return 11;
        case 4096: return 12;
        case 8192: return 13;
        case 16384: return 14;
        case 32768: return 15;
        default: break;
    }
    const int bl = 32 - __builtin_clz((unsigned)bs);
    return bl <= 8 ? 6 : bl <= 16 ? 7 : 0;
}

/* Frame header bytes (CRC-8 included) into h[16]; returns the byte count, or -1 when the
 * frame number needs more than 31 bits (coded_number.py:36-38 ValueError). */
__device__ int frame_header(int64_t fno, int bs, uint8_t* h) {
    const int code = bs_code(bs);
    h[0] = 0xFF;
    h[1] = 0xF8;                /* sync 0b111111111111100 + BlockingStrategy.Fixed (0) */
    h[2] = (uint8_t)(code << 4); /* sample rate: from STREAMINFO (0000) */
    h[3] = 0x10;                /* channels L_R (0001, encoder.py:95), sample size from STREAMINFO, 0 */
    const int bl = fno == 0 ? 0 : 64 - __builtin_clzll((unsigned long long)fno);
    if (bl > 31) return -1;
    const int size = bl <= 7 ? 1 : bl <= 11 ? 2 : bl <= 16 ? 3 : bl <= 21 ? 4 : bl <= 26 ? 5 : 6;
    int k = 4;
    if (size == 1) {
        h[k++] = (uint8_t)fno;
    } else {
        h[k++] = (uint8_t)(((0xFFu << (8 - size)) & 0xFFu) | (uint32_t)((fno >> (6 * (size - 1))) & 0x3F));
        for (int i = size - 2; i >= 0; --i) h[k++] = (uint8_t)(0x80 | ((fno >> (6 * i)) & 0x3F));
    }
    if (code == 6) h[k++] = (uint8_t)(bs - 1);
    if (code == 7) {
        h[k++] = (uint8_t)((bs - 1) >> 8);
        h[k++] = (uint8_t)(bs - 1);
    }
    uint32_t c = 0; /* CRC-8, x^8 + x^2 + x + 1, init 0 (crc.py:18-22) */
    for (int i = 0; i < k; ++i) {
        c ^= h[i];
        for (int b = 0; b < 8; ++b) c = (c & 0x80) ? ((c << 1) ^ 0x07) & 0xFF : (c << 1) & 0xFF;
    }
    h[k++] = (uint8_t)c;
    return k;
}

__device__ __forceinline__ int unit_len(const FrameArgs& a, int64_t u) {
    return u >= a.n_units - a.n_tail_units ? a.tail_len : a.block_len;
}

/* Bits of the subframe up to the first partition (encoder.py:553-627, :766-767). */
__device__ __forceinline__ uint32_t sub_prefix_bits(const flacmi_unit_meta& m, int ss, int q) {
    const bool lpc = m.kind == FLACMI_KIND_LPC;
    return 8u + (uint32_t)m.order * (uint32_t)ss + (lpc ? 9u + (uint32_t)m.ncoefs * (uint32_t)q : 0u) + 6u;
}

/* Written residual bits (partition parameters + Rice codes) from the reference's estimate
 * rice_bits = sum_k [4 + (p_k > 14 ? 5 : 4) + data_k] (encoder.py:714-727):
 *   Rice4Bit: sum_k [4 + data_k]          = rice_bits - 4 n_parts
 *   Rice5Bit: sum_k [5 + data_k]          = rice_bits - 3 n_parts - #{p_k > 14} */
__device__ __forceinline__ int64_t sub_residual_bits(const flacmi_unit_meta& m, int cnt14) {
    return m.coding_method == 5 ? m.rice_bits - 3LL * m.n_parts - cnt14 : m.rice_bits - 4LL * m.n_parts;
}

/* ====================================================================================
 * k_frame_sizes: one wave per frame
 * ==================================================================================== */
__global__ __launch_bounds__(256) void k_frame_sizes(FrameArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= a.n_frames) return;
    const int64_t u0 = f * a.channels;
    const int bs = unit_len(a, u0);
    uint8_t h[16];
    int st = 0;
    const int hb = frame_header(a.first_frame + f, bs, h);
    if (hb < 0) st = (FLACMI_SITE_CODED_NUMBER << 16) | FLACMI_STATUS_VALUE_ERROR;
    int64_t bits = 0;
    for (int c = 0; c < a.channels && st == 0; ++c) {
        const flacmi_unit_meta& m = a.meta[u0 + c];
        if (m.status != 0) {
            st = (m.site << 16) | m.status;
            break;
        }
        if (m.kind == FLACMI_KIND_LPC && ((a.q - 1) & 15) == 15) {
            st = (FLACMI_SITE_LPC_PRECISION << 16) | FLACMI_STATUS_ASSERTION;
            break;
        }
        int cnt = 0;
        if (m.coding_method == 5) {
            const int32_t* rp = a.rice_params + (u0 + c) * a.params_stride;
            for (int k = lane; k < m.n_parts; k += 64) cnt += rp[k] > 14 ? 1 : 0;
            for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
        }
        bits += (int64_t)sub_prefix_bits(m, a.sample_size, a.q) + sub_residual_bits(m, cnt);
    }
    int64_t bytes = 0;
    if (st == 0) {
        bytes = hb + (bits + 7) / 8 + 2;
        if (bytes >= (1LL << kCrcPowLevels)) {
            st = (FLACMI_SITE_FRAME_SIZE << 16) | FLACMI_STATUS_FRAME_TOO_LARGE;
            bytes = 0;
        }
    }
    if (lane == 0) {
        a.offsets[f + 1] = bytes;
        a.status[f] = st;
        if (f == 0) a.offsets[0] = 0;
    }
}

/* ---- exclusive scan of frame sizes (in place on offsets[1..n]) ---------------------- */
constexpr int kScanItems = 8;
constexpr int kScanBlock = 256 * kScanItems;

__device__ __forceinline__ int64_t block_incl_scan(int64_t v, int64_t* sh, int64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == 63) sh[wid] = v;
    __syncthreads();
    int64_t pre = 0, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wid) pre += sh[w];
        tot += sh[w];
    }
    __syncthreads();
    *total = tot;
    return v + pre;
}

__global__ __launch_bounds__(256) void k_scan_local(int64_t* x, int64_t n, int64_t* bsum) {
    __shared__ int64_t sh[4];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanItems;
    int64_t v[kScanItems], s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = base + k < n ? x[base + k] : 0;
        s += v[k];
    }
    int64_t tot;
    const int64_t incl = block_incl_scan(s, sh, &tot);
    int64_t run = incl - s;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        run += v[k];
        if (base + k < n) x[base + k] = run;
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_sums(int64_t* bsum, int64_t nb) {
    __shared__ int64_t sh[4];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += 256) {
        const int64_t i = b0 + threadIdx.x;
        const int64_t v = i < nb ? bsum[i] : 0;
        int64_t tot;
        const int64_t incl = block_incl_scan(v, sh, &tot);
        if (i < nb) bsum[i] = carry + incl - v; /* exclusive */
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void k_scan_add(int64_t* x, int64_t n, const int64_t* bsum) {
    const int64_t base = (int64_t)blockIdx.x * kScanBlock;
    const int64_t add = bsum[blockIdx.x];
    for (int k = threadIdx.x; k < kScanBlock; k += 256)
        if (base + k < n) x[base + k] += add;
}

/* ====================================================================================
 * k_pack
 * ==================================================================================== */
struct CrcTabs {
    const uint16_t* slice; /* [4][256]: T_k[v] = v * x^(16+8k) mod P */
    const uint16_t* pw;    /* [kCrcPowLevels][512]: c -> c * x^(8*2^b) mod P, low byte | high byte */
};

__device__ __forceinline__ uint32_t crc16_mulpow(uint32_t c, int64_t d, const uint16_t* __restrict__ pw) {
    for (int b = 0; d != 0 && c != 0; ++b, d >>= 1)
        if (d & 1) c = (uint32_t)pw[b * 512 + (c & 0xFF)] ^ (uint32_t)pw[b * 512 + 256 + (c >> 8)];
    return c;
}

/* OR the w-bit value v (right-aligned, 1 <= w <= 64) at aligned bit position pos into the
 * window covering aligned words [wb, wb + kWinWords); parts outside are skipped. */
__device__ __forceinline__ void win_or(uint32_t* win, uint32_t wb, uint32_t pos, uint64_t v, int w) {
    const uint32_t end = pos + (uint32_t)w;
    uint32_t lo = pos > wb * 32u ? pos : wb * 32u;
    const uint32_t wend_all = (wb + kWinWords) * 32u;
    const uint32_t hi = end < wend_all ? end : wend_all;
    while (lo < hi) {
        const uint32_t word = lo >> 5;
        const uint32_t we = (word + 1) * 32u;
        const uint32_t pe = hi < we ? hi : we;
        const int nb = (int)(pe - lo);
        const uint32_t piece = (uint32_t)((v >> (end - pe)) & ((nb == 64 ? 0ull : (1ull << nb)) - 1ull));
        atomicOr(&win[word - wb], piece << (32 - (int)(lo & 31) - nb));
        lo = pe;
    }
}

/* Flush window words [0, nw) (aligned words wb..wb+nw) to the output: CRC-16 contributions
 * of the bytes in [F, E) first, then (final) the CRC itself at E, then the stores. */
__device__ void win_flush(const FrameArgs& a, uint32_t* win, const uint16_t* ct, uint32_t wb, int nw, bool final,
                          int64_t F, int64_t Fend, uint32_t& crc_acc, uint32_t* red) {
    const int tid = threadIdx.x, NT = blockDim.x;
    const int64_t E = Fend - 2;
    const int64_t gw0 = (F >> 2) + wb; /* output word of window word 0 */
    {
        const int wpt = (nw + NT - 1) / NT;
        const int k0 = tid * wpt, k1 = k0 + wpt < nw ? k0 + wpt : nw;
        uint32_t c = 0;
        int64_t R = -1;
        for (int k = k0; k < k1; ++k) {
            const int64_t gb = 4 * (gw0 + k);
            const uint32_t w = win[k];
            if (gb >= F && gb + 4 <= E) {
                c = (uint32_t)ct[3 * 256 + ((c >> 8) ^ (w >> 24))] ^ (uint32_t)ct[2 * 256 + ((c ^ (w >> 16)) & 0xFF)] ^
                    (uint32_t)ct[256 + ((w >> 8) & 0xFF)] ^ (uint32_t)ct[w & 0xFF];
                R = gb + 4;
            } else {
                for (int j = 0; j < 4; ++j) {
                    const int64_t B = gb + j;
                    if (B >= F && B < E) {
                        c = ((c << 8) & 0xFFFF) ^ (uint32_t)ct[(c >> 8) ^ ((w >> (24 - 8 * j)) & 0xFF)];
                        R = B + 1;
                    }
                }
            }
        }
        if (R >= 0) crc_acc ^= crc16_mulpow(c, E - R, a.crc_pow);
    }
    __syncthreads(); /* every CRC read of the window precedes the stores below */
    if (final) {
        uint32_t v = crc_acc;
        for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o);
        if ((tid & 63) == 0) red[tid >> 6] = v;
        __syncthreads();
        if (tid == 0) {
            uint32_t crc = 0;
            for (int w2 = 0; w2 < NT / 64; ++w2) crc ^= red[w2];
            const uint32_t pos = (uint32_t)(8 * (F & 3) + 8 * (E - F));
            win_or(win, wb, pos, crc & 0xFFFF, 16);
        }
        __syncthreads();
    }
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out);
    for (int k = tid; k < nw; k += NT) {
        const int64_t g = gw0 + k;
        const uint32_t w = win[k];
        if (4 * g >= F && 4 * g + 4 <= Fend) {
            out32[g] = __builtin_bswap32(w);
        } else {
            for (int j = 0; j < 4; ++j) {
                const int64_t B = 4 * g + j;
                if (B >= F && B < Fend) a.out[B] = (uint8_t)(w >> (24 - 8 * j));
            }
        }
        win[k] = 0;
    }
    __syncthreads();
}

/* k_pack32 takes a frame when it fits one LDS window (with its alignment offset and the
 * CRC) and every partition holds at least 8 values (a chunk of 8 meets at most one
 * partition boundary); the launch guarantees 32-bit residuals and <= kMaxC chunks per
 * thread. */
constexpr int kMaxC = 4;
__device__ __forceinline__ bool pack32_frame_ok(const FrameArgs& a, int64_t f, int ww) {
    const int64_t bytes = a.offsets[f + 1] - a.offsets[f];
    if (bytes + 8 > 4LL * ww) return false;
    for (int c = 0; c < a.channels; ++c) {
        const int64_t u = f * a.channels + c;
        if ((unit_len(a, u) >> a.meta[u].part_order) < 8) return false;
    }
    return true;
}

template <typename ZT>
__device__ __forceinline__ void pack_frame(const FrameArgs& a, const int64_t f) {
    __shared__ uint32_t win[kWinWords];
    __shared__ uint16_t ct[4 * 256];
    __shared__ uint8_t hdr[16];
    __shared__ uint32_t sub_start[9];
    __shared__ int32_t cnt14[8];
    __shared__ uint32_t red[8];
    __shared__ int hb_s;
    const int tid = threadIdx.x, NT = blockDim.x, lane = tid & 63, wid = tid >> 6;
    if (a.status[f] != 0) return;
    const int64_t F = a.offsets[f], Fend = a.offsets[f + 1];
    const int64_t u0 = f * a.channels;
    const int C = a.channels;
    for (int i = tid; i < 4 * 256; i += NT) ct[i] = a.crc_slice[i];
    for (int i = tid; i < kWinWords; i += NT) win[i] = 0;
    if (tid < 8) cnt14[tid] = 0;
    if (tid == 0) hb_s = frame_header(a.first_frame + f, unit_len(a, u0), hdr);
    __syncthreads();
    for (int c = 0; c < C; ++c) {
        const flacmi_unit_meta& m = a.meta[u0 + c];
        if (m.coding_method == 5) {
            const int32_t* rp = a.rice_params + (u0 + c) * a.params_stride;
            int cnt = 0;
            for (int k = tid; k < m.n_parts; k += NT) cnt += rp[k] > 14 ? 1 : 0;
            if (cnt) atomicAdd(&cnt14[c], cnt);
        }
    }
    __syncthreads();
    const int hb = hb_s;
    const uint32_t A = (uint32_t)(8 * (F & 3)); /* aligned bit of the frame's first bit */
    if (tid == 0) {
        uint32_t s = A + 8u * (uint32_t)hb;
        for (int c = 0; c < C; ++c) {
            const flacmi_unit_meta& m = a.meta[u0 + c];
            sub_start[c] = s;
            s += sub_prefix_bits(m, a.sample_size, a.q) + (uint32_t)sub_residual_bits(m, cnt14[c]);
        }
        sub_start[C] = s;
    }
    __syncthreads();

    uint32_t wb = 0, crc_acc = 0;
    /* run `body` until the segment ending at aligned bit seg_end is in the window; full
     * windows are flushed in between (uniform control flow) */
    auto segment = [&](uint32_t seg_end, auto&& body) __attribute__((always_inline)) {
        while (true) {
            body();
            if (seg_end <= (wb + kWinWords) * 32u) break;
            __syncthreads();
            win_flush(a, win, ct, wb, kWinWords, false, F, Fend, crc_acc, red);
            wb += kWinWords;
        }
    };
    /* frame header: byte fields */
    segment(A + 8u * hb, [&]() {
        if (tid < hb) win_or(win, wb, A + 8u * tid, hdr[tid], 8);
    });
    const int ss = a.sample_size, q = a.q;
    for (int c = 0; c < C; ++c) {
        const int64_t u = u0 + c;
        const flacmi_unit_meta& m = a.meta[u];
        const int n = unit_len(a, u);
        const int order = m.order, ncoefs = m.ncoefs, method = m.coding_method;
        const bool lpc = m.kind == FLACMI_KIND_LPC;
        const uint32_t s0 = sub_start[c];
        const uint32_t pre = sub_prefix_bits(m, ss, q);
        /* subframe header, warm-up, LPC fields, residual header: field t per thread */
        const int nfields = 1 + order + (lpc ? 2 + ncoefs : 0) + 2;
        segment(s0 + pre, [&]() {
            for (int t = tid; t < nfields; t += NT) {
                uint32_t pos;
                uint64_t v;
                int w;
                if (t == 0) {
                    pos = s0;
                    v = lpc ? (uint64_t)((0x20 | (order - 1)) << 1) : (uint64_t)((0x08 | order) << 1);
                    w = 8;
                } else if (t <= order) {
                    const int j = t - 1;
                    const int64_t x = a.sample_bytes == 2 ? (int64_t)((const int16_t*)a.samples)[u * a.stride + j]
                                                          : (int64_t)((const int32_t*)a.samples)[u * a.stride + j];
                    pos = s0 + 8 + (uint32_t)j * ss;
                    v = (uint64_t)x & (ss == 64 ? ~0ull : ((1ull << ss) - 1));
                    w = ss;
                } else {
                    const uint32_t b = s0 + 8 + (uint32_t)order * ss;
                    const int t2 = t - 1 - order;
                    if (lpc && t2 == 0) {
                        pos = b;
                        v = (uint64_t)((q - 1) & 15);
                        w = 4;
                    } else if (lpc && t2 == 1) {
                        pos = b + 4;
                        v = (uint64_t)(m.shift & 31);
                        w = 5;
                    } else if (lpc && t2 < 2 + ncoefs) {
                        const int j = t2 - 2;
                        pos = b + 9 + (uint32_t)j * q;
                        v = (uint64_t)(int64_t)m.coefs[j] & ((1ull << q) - 1);
                        w = q;
                    } else {
                        const int t3 = t2 - (lpc ? 2 + ncoefs : 0);
                        const uint32_t b2 = b + (lpc ? 9u + (uint32_t)ncoefs * q : 0u);
                        if (t3 == 0) {
                            pos = b2;
                            v = method == 5 ? 1 : 0;
                            w = 2;
                        } else {
                            pos = b2 + 2;
                            v = (uint64_t)(m.part_order & 15);
                            w = 4;
                        }
                    }
                }
                win_or(win, wb, pos, v, w);
            }
        });
        /* partitions: parameter + Rice codes, 8 residual values per thread per tile */
        const int ps = n >> m.part_order;
        const int32_t* __restrict__ rp = a.rice_params + u * a.params_stride;
        const ZT* __restrict__ zrow = reinterpret_cast<const ZT*>(a.residual) + u * a.residual_stride;
        const int nch = (n + 7) >> 3;
        const uint64_t pmask_m = (1ull << method) - 1;
        uint32_t tile_base = s0 + pre;
        for (int c0 = 0; c0 < nch; c0 += NT) {
            const int ch = c0 + tid;
            const int i0 = 8 * ch;
            ZT z[8];
            int pp[8];
            uint32_t len[8];
            uint32_t tsum = 0;
            /* partition of each value: one division per chunk; with ps >= 8 a chunk meets
             * at most one partition boundary */
            const int part0 = i0 / ps;
            const int bnd = (part0 + 1) * ps;
            int pA = 0, pB = 0;
            if (ch < nch && ps >= 8) {
                pA = rp[part0 < m.n_parts ? part0 : m.n_parts - 1];
                pB = (bnd < n && bnd <= i0 + 7) ? rp[part0 + 1] : pA;
            }
            int part = part0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k;
                const bool valid = ch < nch && i >= order && i < n;
                int p;
                if (ps >= 8) {
                    p = i >= bnd ? pB : pA;
                } else {
                    while ((part + 1) * ps <= i) ++part;
                    p = valid ? rp[part] : 0;
                }
                p = valid ? p : 0;
                z[k] = valid ? zrow[i] : (ZT)0;
                const bool first = valid && (i == order || (i > order && (i == bnd || i == part0 * ps ||
                                                                          (ps < 8 && i == part * ps))));
                pp[k] = first ? p | 0x100 : p;
                const uint32_t qv = p >= (int)(8 * sizeof(ZT)) ? 0u : (uint32_t)(z[k] >> p);
                len[k] = valid ? (first ? (uint32_t)method : 0u) + qv + 1u + (uint32_t)p : 0u;
                tsum += len[k];
            }
            /* workgroup exclusive scan of tsum */
            uint32_t v = tsum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += t;
            }
            if (lane == 63) red[wid] = v;
            __syncthreads();
            uint32_t pre_w = 0, tot = 0;
            for (int w2 = 0; w2 < NT / 64; ++w2) {
                const uint32_t s = red[w2];
                if (w2 < wid) pre_w += s;
                tot += s;
            }
            __syncthreads();
            const uint32_t tstart = tile_base + pre_w + v - tsum;
            if constexpr (sizeof(ZT) == 4) {
                /* this thread's codes are contiguous: assemble them in a 64-bit buffer and
                 * OR whole words into the window (its first and last word are shared) */
                segment(tile_base + tot, [&]() {
                    const uint32_t wlo = wb, whi = wb + kWinWords;
                    uint32_t pos = tstart, widx = tstart >> 5;
                    uint64_t acc = 0;
                    auto emit = [&](uint32_t wi, uint32_t val) __attribute__((always_inline)) {
                        if (val != 0 && wi >= wlo && wi < whi) atomicOr(&win[wi - wlo], val);
                    };
                    /* v right-aligned, 1 <= w <= 32; keeps pos - 32*widx in [0, 32) */
                    auto put = [&](uint32_t val, int w) __attribute__((always_inline)) {
                        const int off = (int)(pos - 32u * widx);
                        acc |= (uint64_t)val << (64 - off - w);
                        pos += (uint32_t)w;
                        if (pos - 32u * widx >= 32u) {
                            emit(widx, (uint32_t)(acc >> 32));
                            acc <<= 32;
                            ++widx;
                        }
                    };
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if (len[k] != 0) {
                            const int p = pp[k] & 0xFF;
                            if (pp[k] & 0x100) put((uint32_t)p & (uint32_t)pmask_m, method);
                            const uint32_t zk = (uint32_t)z[k];
                            const uint32_t qv = p >= 32 ? 0u : zk >> p;
                            if (qv != 0) { /* unary zeros */
                                pos += qv;
                                if (pos - 32u * widx >= 32u) {
                                    emit(widx, (uint32_t)(acc >> 32));
                                    acc = 0;
                                    widx = pos >> 5;
                                }
                            }
                            /* the one and the p low bits: p + 1 <= 32 bits */
                            const uint32_t lowm = p >= 32 ? 0xFFFFFFFFu : ((1u << p) - 1u);
                            if (p >= 32) { /* not reachable for 32-bit values (p <= 31); kept exact */
                                put(1u, 1);
                                pos += (uint32_t)(p - 32);
                                if (pos - 32u * widx >= 32u) {
                                    emit(widx, (uint32_t)(acc >> 32));
                                    acc = 0;
                                    widx = pos >> 5;
                                }
                                put(zk, 32);
                            } else {
                                put((1u << p) | (zk & lowm), p + 1);
                            }
                        }
                    }
                    if (pos != 32u * widx) emit(widx, (uint32_t)(acc >> 32));
                });
            } else {
                segment(tile_base + tot, [&]() {
                    uint32_t pos = tstart;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if (len[k] != 0) {
                            const int p = pp[k] & 0xFF;
                            uint32_t at = pos;
                            if (pp[k] & 0x100) {
                                win_or(win, wb, at, (uint64_t)p & pmask_m, method);
                                at += (uint32_t)method;
                            }
                            const uint32_t qv = p >= (int)(8 * sizeof(ZT)) ? 0u : (uint32_t)(z[k] >> p);
                            const uint64_t val = (1ull << p) | ((uint64_t)z[k] & ((1ull << p) - 1));
                            win_or(win, wb, at + qv, val, p + 1);
                            pos += len[k];
                        }
                    }
                });
            }
            tile_base += tot;
        }
    }
    __syncthreads();
    /* padding is already zero; the CRC-16 goes at byte E = Fend - 2 */
    const uint32_t endbit = (uint32_t)(8 * (F & 3) + 8 * (Fend - F));
    /* the CRC bytes must land in the final window */
    while (endbit > (wb + kWinWords) * 32u) {
        win_flush(a, win, ct, wb, kWinWords, false, F, Fend, crc_acc, red);
        wb += kWinWords;
    }
    const int nw = (int)((endbit + 31) / 32 - wb);
    win_flush(a, win, ct, wb, nw, true, F, Fend, crc_acc, red);
}

/* General frame writer: every frame (pack_split = 0), or, after k_pack32, the frames it
 * listed (grid-stride over the list; an empty list costs one short launch). */
template <typename ZT>
__global__ __launch_bounds__(kPackThreads) void k_pack(FrameArgs a) {
    if (a.offsets[a.n_frames] > a.capacity) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            a.status[0] = (FLACMI_SITE_FRAME_SIZE << 16) | FLACMI_STATUS_FRAME_TOO_LARGE;
        return;
    }
    const int64_t cnt = a.pack_split ? (int64_t)*a.slow_count : (int64_t)blockIdx.x + 1;
    for (int64_t idx = blockIdx.x; idx < cnt; idx += gridDim.x) { /* one call site: inlined once */
        pack_frame<ZT>(a, a.pack_split ? a.slow_list[idx] : idx);
        __syncthreads(); /* LDS reuse by the next frame */
    }
}

/* ====================================================================================
 * k_pack32: the frame writer for frames that fit one LDS window (32-bit residuals).
 *
 * One workgroup per frame.  Thread t owns a CONTIGUOUS run of 8-value chunks of each
 * subframe (kMaxC at most, kept in registers), so one workgroup scan per subframe gives
 * every thread the bit position of its run; the thread assembles its codes in a 64-bit
 * register and ORs whole 32-bit words into the window (only the first and last word of a
 * run are shared with a neighbour).  CRC-16: thread t folds a 4-byte-multiple segment of
 * the frame ending at E - S*(NT-1-t) (E = the CRC position; window words read with a byte
 * funnel shift, bytes before the frame treated as the leading zeros they are to a CRC that
 * starts at 0), shifts it to E with the x^(8*2^b) tables and the workgroup XORs the
 * shares.  The frame is stored with 16-byte stores (dword / byte stores at its two ends).
 * ==================================================================================== */
/* k_pack32: the w-bit field val (1 <= w <= 32) ORed into the window at bit P, one or two
 * words (bit 31 of a window word is its first bit; the second OR is zero unless the field
 * straddles a word boundary) */
__device__ __forceinline__ void or_bits(uint32_t* win, uint32_t P, uint32_t val, uint32_t w) {
    const uint64_t t = (uint64_t)val << (64u - (P & 31u) - w);
    uint32_t* wp = win + (P >> 5);
    atomicOr(wp, (uint32_t)(t >> 32));
    atomicOr(wp + 1, (uint32_t)t);
}

/* MAXC: chunks per thread the launch guarantees (2..kMaxC): fewer registers, more frames in
 * flight per CU.  WW: window words (frames larger go to k_pack by list); WPE: occupancy floor
 * in waves a SIMD.  A 3072-word window (14.3 KB of LDS) lets 10 workgroups share a CU, so
 * the floor of 7 waves (72 VGPRs, no spills) is reachable; the 16 KB window capped it at 8
 * workgroups, 6 waves a SIMD for 192-thread groups. */
template <int MAXC, int WW, int WPE>
__global__ __launch_bounds__(kPackThreads) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_pack32(FrameArgs a) {
    __shared__ uint32_t win[WW];
    __shared__ __align__(16) uint16_t ct[4 * 256];
    __shared__ uint8_t hdr[16];
    __shared__ uint32_t sub_start[9];
    __shared__ int32_t cnt14[8];
    __shared__ uint32_t red[kPackThreads / 64];
    __shared__ int hb_s;
    const int tid = threadIdx.x, NT = blockDim.x, lane = tid & 63, wid = tid >> 6;
    const int64_t f = blockIdx.x;
    /* one dword of every 128-byte line of the first subframe's residual row, loaded before
     * anything is checked: the row's HBM round trip then overlaps the chain of small dependent
     * loads below (offsets, status, meta, parameters), and the chunk loads later hit L2 (the
     * value itself is never used) */
    uint32_t touch = 0;
    if (!(a.ablate & 64)) {
        const int64_t u = f * a.channels;
        const int lines = (unit_len(a, u) * 4 + 127) >> 7;
        const uint32_t* __restrict__ zrow = reinterpret_cast<const uint32_t*>(a.residual) + u * a.residual_stride;
        touch = zrow[32 * min(tid, lines - 1)];
    }
    if (a.offsets[a.n_frames] > a.capacity) return; /* k_pack reports it */
    if (a.status[f] != 0) return;
    if (!pack32_frame_ok(a, f, WW)) { /* k_pack writes it */
        if (threadIdx.x == 0) a.slow_list[atomicAdd(a.slow_count, 1ull)] = f;
        return;
    }
    const int64_t F = a.offsets[f], Fend = a.offsets[f + 1];
    const int64_t u0 = f * a.channels;
    const int C = a.channels;
    const uint32_t A = (uint32_t)(8 * (F & 3)); /* aligned bit of the frame's first bit */
    const int nwf = (int)(((F & 3) + (Fend - F) + 3) >> 2); /* window words of the frame */
    /* the 2 KB of CRC slice tables as 128 16-byte loads (not 1024 2-byte ones) */
    for (int i = tid; i < 128; i += NT) reinterpret_cast<uint4*>(ct)[i] = reinterpret_cast<const uint4*>(a.crc_slice)[i];
    for (int i = tid; i < nwf; i += NT) win[i] = 0;
    if (tid < 8) cnt14[tid] = 0;
    if (tid == 0) hb_s = frame_header(a.first_frame + f, unit_len(a, u0), hdr);
    __syncthreads();
    for (int c = 0; c < C; ++c) {
        const flacmi_unit_meta& m = a.meta[u0 + c];
        if (m.coding_method == 5) {
            const int32_t* rp = a.rice_params + (u0 + c) * a.params_stride;
            int cnt = 0;
            for (int k = tid; k < m.n_parts; k += NT) cnt += rp[k] > 14 ? 1 : 0;
            if (cnt) atomicAdd(&cnt14[c], cnt);
        }
    }
    __syncthreads();
    const int hb = hb_s;
    if (tid == 0) {
        uint32_t s = A + 8u * (uint32_t)hb;
        for (int c = 0; c < C; ++c) {
            const flacmi_unit_meta& m = a.meta[u0 + c];
            sub_start[c] = s;
            s += sub_prefix_bits(m, a.sample_size, a.q) + (uint32_t)sub_residual_bits(m, cnt14[c]);
        }
        sub_start[C] = s;
    }
    if (tid < hb) win_or(win, 0, A + 8u * tid, hdr[tid], 8);
    __syncthreads();

    const int ss = a.sample_size, q = a.q;
    for (int c = 0; c < C; ++c) {
        const int64_t u = u0 + c;
        const flacmi_unit_meta& m = a.meta[u];
        const int n = unit_len(a, u);
        const int order = m.order, ncoefs = m.ncoefs, method = m.coding_method;
        const bool lpc = m.kind == FLACMI_KIND_LPC;
        const uint32_t s0 = sub_start[c];
        const uint32_t pre = sub_prefix_bits(m, ss, q);
        /* subframe header, warm-up, LPC fields, residual header: field t per thread */
        const int nfields = 1 + order + (lpc ? 2 + ncoefs : 0) + 2;
        for (int t = tid; t < nfields; t += NT) {
            uint32_t pos;
            uint64_t v;
            int w;
            const uint32_t b = s0 + 8 + (uint32_t)order * ss;
            const int t2 = t - 1 - order;
            if (t == 0) {
                pos = s0;
                v = lpc ? (uint64_t)((0x20 | (order - 1)) << 1) : (uint64_t)((0x08 | order) << 1);
                w = 8;
            } else if (t <= order) {
                const int j = t - 1;
                const int64_t x = a.sample_bytes == 2 ? (int64_t)((const int16_t*)a.samples)[u * a.stride + j]
                                                      : (int64_t)((const int32_t*)a.samples)[u * a.stride + j];
                pos = s0 + 8 + (uint32_t)j * ss;
                v = (uint64_t)x & (ss == 64 ? ~0ull : ((1ull << ss) - 1));
                w = ss;
            } else if (lpc && t2 == 0) {
                pos = b;
                v = (uint64_t)((q - 1) & 15);
                w = 4;
            } else if (lpc && t2 == 1) {
                pos = b + 4;
                v = (uint64_t)(m.shift & 31);
                w = 5;
            } else if (lpc && t2 < 2 + ncoefs) {
                const int j = t2 - 2;
                pos = b + 9 + (uint32_t)j * q;
                v = (uint64_t)(int64_t)m.coefs[j] & ((1ull << q) - 1);
                w = q;
            } else {
                const int t3 = t2 - (lpc ? 2 + ncoefs : 0);
                const uint32_t b2 = b + (lpc ? 9u + (uint32_t)ncoefs * q : 0u);
                pos = t3 == 0 ? b2 : b2 + 2;
                v = t3 == 0 ? (method == 5 ? 1 : 0) : (uint64_t)(m.part_order & 15);
                w = t3 == 0 ? 2 : 4;
            }
            win_or(win, 0, pos, v, w);
        }
        /* residual: this thread's chunks [k0, k1) */
        const int ps = n >> m.part_order;
        const int32_t* __restrict__ rp = a.rice_params + u * a.params_stride;
        const uint32_t* __restrict__ zrow = reinterpret_cast<const uint32_t*>(a.residual) + u * a.residual_stride;
        const int nch = (n + 7) >> 3;
        const int cpt = (nch + NT - 1) / NT;
        const int k0 = tid * cpt, k1 = min(k0 + cpt, nch);
        uint32_t z[MAXC][8];
        int pa[MAXC], pb[MAXC], bnd[MAXC], pt0[MAXC];
        uint32_t tsum = 0;
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
            const int k = k0 + j;
            const int i0 = 8 * k;
            pa[j] = pb[j] = 0;
            bnd[j] = 1 << 30;
            if (k < k1) {
                uint4 v0{0, 0, 0, 0}, v1{0, 0, 0, 0};
                if (a.ablate & 32) { /* ablation 32: no residual loads (timing only) */
                } else if (i0 + 8 <= n) {
                    v0 = *reinterpret_cast<const uint4*>(zrow + i0);
                    v1 = *reinterpret_cast<const uint4*>(zrow + i0 + 4);
                } else { /* the row's last chunk: no reads past its end */
                    v0 = uint4{zrow[i0], i0 + 1 < n ? zrow[i0 + 1] : 0u, i0 + 2 < n ? zrow[i0 + 2] : 0u,
                               i0 + 3 < n ? zrow[i0 + 3] : 0u};
                    v1 = uint4{i0 + 4 < n ? zrow[i0 + 4] : 0u, i0 + 5 < n ? zrow[i0 + 5] : 0u,
                               i0 + 6 < n ? zrow[i0 + 6] : 0u, i0 + 7 < n ? zrow[i0 + 7] : 0u};
                }
                if (j == 0 && c == 0 && (a.ablate & 128)) v0.x ^= touch; /* never set: keeps the touch load */
                z[j][0] = v0.x; z[j][1] = v0.y; z[j][2] = v0.z; z[j][3] = v0.w;
                z[j][4] = v1.x; z[j][5] = v1.y; z[j][6] = v1.z; z[j][7] = v1.w;
                const int part0 = i0 / ps;
                pt0[j] = part0;
                const int b1 = (part0 + 1) * ps;
                pa[j] = rp[part0];
                pb[j] = (b1 < n && b1 <= i0 + 7) ? rp[part0 + 1] : pa[j];
                bnd[j] = b1;
                if (i0 > order && i0 + 8 <= n && b1 >= i0 + 8) { /* one partition, every value coded */
                    const int p = pa[j];
                    uint32_t q = 0;
#pragma unroll
                    for (int e = 0; e < 8; ++e) q += z[j][e] >> p;
                    tsum += q + 8u * (uint32_t)(p + 1) + (i0 == part0 * ps ? (uint32_t)method : 0u);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int i = i0 + e;
                        const int p = i >= b1 ? pb[j] : pa[j];
                        const bool valid = i >= order && i < n;
                        const bool first = i == order || (i > order && (i == b1 || i == part0 * ps));
                        tsum += valid ? (first ? (uint32_t)method : 0u) + (z[j][e] >> p) + 1u + (uint32_t)p : 0u;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) z[j][e] = 0;
            }
        }
        /* workgroup exclusive scan of tsum */
        uint32_t v = tsum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)v, o);
            if (lane >= o) v += t;
        }
        if (lane == 63) red[wid] = v;
        __syncthreads();
        uint32_t pre_w = 0;
        for (int w2 = 0; w2 < wid; ++w2) pre_w += red[w2];
        uint32_t pos = s0 + pre + pre_w + v - tsum;
        /* Every field lands in the zeroed window by LDS ORs at its bit position: a code's q unary
         * zeros need no write, its terminating 1 and p low bits (<= 31 bits) take one or two ORs,
         * and so does a partition's parameter.  No per-thread bit accumulator and no branch on
         * where a word fills (round 6; the accumulator's emit branches and 64-bit shifts cost
         * about 28 VALU per value). */
        const uint32_t pmask_m = (1u << method) - 1u;
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
            const int k = k0 + j;
            if (k < k1 && !(a.ablate & 2)) {
                const int i0 = 8 * k;
                const int part0 = pt0[j];
                /* a chunk inside (order, n) whose values share one partition (the common case): at
                 * most its first value opens a partition, so the parameter goes in before the
                 * values, which then run straight-line */
                if (i0 > order && i0 + 8 <= n && bnd[j] >= i0 + 8) {
                    const int p = pa[j];
                    if (i0 == part0 * ps) {
                        or_bits(win, pos, (uint32_t)p & pmask_m, (uint32_t)method);
                        pos += (uint32_t)method;
                    }
                    const uint32_t one = 1u << p, wc = (uint32_t)p + 1u;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const uint32_t zk = z[j][e];
                        const uint32_t P = pos + (zk >> p);
                        or_bits(win, P, one | (zk & (one - 1u)), wc);
                        pos = P + wc;
                    }
                } else { /* the warm-up's chunk, the unit's end, a partition boundary inside */
#pragma unroll 1
                    for (int e = 0; e < 8; ++e) {
                        uint32_t zk = z[j][0];
#pragma unroll
                        for (int e2 = 1; e2 < 8; ++e2) zk = e == e2 ? z[j][e2] : zk;
                        const int i = i0 + e;
                        if (i >= order && i < n) {
                            const int p = i >= bnd[j] ? pb[j] : pa[j];
                            if (i == order || i == bnd[j] || i == part0 * ps) {
                                or_bits(win, pos, (uint32_t)p & pmask_m, (uint32_t)method);
                                pos += (uint32_t)method;
                            }
                            const uint32_t P = pos + (zk >> p);
                            or_bits(win, P, (1u << p) | (zk & ((1u << p) - 1u)), (uint32_t)p + 1u); /* p <= 30 */
                            pos = P + (uint32_t)p + 1u;
                        }
                    }
                }
            }
        }
        __syncthreads(); /* red[] reuse by the next subframe's scan */
    }

    /* CRC-16 of bytes [F, E), E = Fend - 2.  Window byte r is frame byte F - (F & 3) + r; the
     * bytes before F are zero, which a CRC that starts at 0 ignores.  The nfull whole window
     * words before E are cut into NT equal segments of spw words (a power of two) that END at
     * word nfull, so thread t's segment lies m = NT - 1 - t segments before it (the first ones
     * reach below word 0: zeros).  Each thread folds its segment's words (one aligned LDS read
     * each), then the shares combine in a tree: at level l the earlier block is shifted by the
     * later block's 2^l segments, a multiplication by x^(8 * 4 spw 2^l), which is one level of
     * the x^(8 2^b) tables, the same for every lane.  Thread 0 adds the waves, then shifts the
     * whole by the 0..3 bytes between word nfull and E and folds those bytes. */
    const int64_t E = Fend - 2;
    const int64_t Fa = F & ~3LL;
    {
        const int nfull = (int)((E - Fa) >> 2);
        int ls = 0;
        while ((NT << ls) < nfull) ++ls;
        const int spw = 1 << ls;
        const int w1 = nfull - (NT - 1 - tid) * spw, w0 = w1 - spw;
        const uint16_t* __restrict__ pw = a.crc_pow;
        auto mulx = [&](uint32_t c, int bl) __attribute__((always_inline)) { /* c * x^(8 * 2^bl) mod P */
            return (uint32_t)pw[bl * 512 + (c & 0xFF)] ^ (uint32_t)pw[bl * 512 + 256 + (c >> 8)];
        };
        uint32_t crc = 0;
        if (!(a.ablate & 4)) { /* ablation 4: no CRC fold (timing only) */
            for (int k = max(w0, 0); k < w1; ++k) {
                const uint32_t w = win[k];
                crc = (uint32_t)ct[3 * 256 + ((crc >> 8) ^ (w >> 24))] ^ (uint32_t)ct[2 * 256 + ((crc ^ (w >> 16)) & 0xFF)] ^
                      (uint32_t)ct[256 + ((w >> 8) & 0xFF)] ^ (uint32_t)ct[w & 0xFF];
            }
        }
        if (!(a.ablate & 1)) { /* ablation 1: no shift (timing only) */
#pragma unroll
            for (int l = 0; l < 6; ++l) {
                const uint32_t other = (uint32_t)__shfl_xor((int)crc, 1 << l);
                const bool right = (lane >> l) & 1;
                crc = mulx(right ? other : crc, ls + 2 + l) ^ (right ? crc : other);
            }
        } else {
            for (int o2 = 32; o2 >= 1; o2 >>= 1) crc ^= (uint32_t)__shfl_xor((int)crc, o2);
        }
        if (lane == 0) red[wid] = crc;
        __syncthreads();
        if (tid == 0) {
            uint32_t x = 0;
            for (int w2 = 0; w2 < NT / 64; ++w2) x = (w2 ? mulx(x, ls + 8) : 0u) ^ red[w2]; /* 64 segments a wave */
            const int tail = (int)(E - Fa) - 4 * nfull;
            for (int j = 0; j < tail; ++j) x = ((x << 8) & 0xFFFF) ^ (uint32_t)ct[(x >> 8) ^ ((win[nfull] >> (24 - 8 * j)) & 0xFF)];
            win_or(win, 0, (uint32_t)(8 * (F & 3) + 8 * (E - F)), x & 0xFFFF, 16);
        }
        __syncthreads();
    }

    /* store: window word k is output word (F >> 2) + k */
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out);
    const int64_t g0 = F >> 2;
    const int64_t gf = (F + 3) >> 2;   /* first word wholly inside the frame */
    const int64_t ge = Fend >> 2;      /* words [gf, ge) are wholly inside */
    if (tid < 4) { /* partial words at both ends: byte stores */
        const int64_t g = tid < 2 ? g0 : ge;
        const int j = tid & 1 ? 2 : 0;
        for (int jj = j; jj < j + 2; ++jj) {
            const int64_t B = 4 * g + jj;
            if (B >= F && B < Fend && !(g >= gf && g < ge)) a.out[B] = (uint8_t)(win[g - g0] >> (24 - 8 * jj));
        }
    }
    if (gf < ge && !(a.ablate & 16)) { /* ablation 16: no stores of the frame's body (timing only) */
        const int64_t mis = (int64_t)(((uintptr_t)a.out >> 2) & 3); /* out is 4-byte aligned */
        const int64_t ga = ((gf + mis + 3) & ~3LL) - mis; /* 16-byte aligned output words [ga, gz) */
        const int64_t gz = ((ge + mis) & ~3LL) - mis;
        if (ga < gz) {
            for (int64_t g = ga + 4 * tid; g < gz; g += 4 * NT) {
                const int64_t k = g - g0;
                uint4 v{__builtin_bswap32(win[k]), __builtin_bswap32(win[k + 1]), __builtin_bswap32(win[k + 2]),
                        __builtin_bswap32(win[k + 3])};
                *reinterpret_cast<uint4*>(out32 + g) = v;
            }
            if (tid < 3 && gf + tid < ga) out32[gf + tid] = __builtin_bswap32(win[gf + tid - g0]);
            if (tid >= 4 && tid < 7 && gz + (tid - 4) < ge) out32[gz + tid - 4] = __builtin_bswap32(win[gz + tid - 4 - g0]);
        } else if (tid < 4) {
            for (int64_t g = gf + tid; g < ge; g += 4) out32[g] = __builtin_bswap32(win[g - g0]);
        }
    }
}

/* ====================================================================================
 * k_packw: the frame writer for frames of more than kMaxC chunks a thread (config 3's
 * 16384-sample stereo frames, 89 KB each; 32-bit residuals, partitions of >= 8 values).
 *
 * k_pack32's placement run tile after tile: a tile is NT * MAXC chunks, one workgroup scan
 * gives each thread the bit position of its contiguous run, and every code is ORed into
 * LDS at its bit position.  The LDS window is a ring of RW words; window bit 0 is the
 * 16-byte aligned output address at or below the frame's first byte.  Bits below a
 * segment's end (the frame header, a subframe's header fields, a tile) are final, so after
 * each segment the whole 2 NT-word chunks below it leave the ring: thread t takes words 2t
 * and 2t+1 of the chunk (one 8-byte LDS read, one 8-byte store, zeroed behind), folds their
 * CRC-16 and adds it to its own running CRC multiplied by x^(8 * 8 NT) (the chunk length;
 * one table in LDS).  At the frame's end a lane tree turns the running CRCs into the CRC
 * of everything that left, k_pack32's end fold takes the last < 2 NT words, and the two
 * are joined with one x^(8d) multiplication.  A segment that would overrun the ring writes
 * what fits (ORs outside [fl, fl + RW) are skipped), the full ring leaves, and the segment
 * runs again: ORs are idempotent.  The default build is one wave a workgroup (NT = 64, a
 * 4 KB ring), so its barriers are one wave's.  The general k_pack flushes a whole window at
 * a time with a per-thread x^(8d) shift from global tables (17 dependent loads a flush) and
 * one-value-at-a-time accumulators; this kernel is its replacement for the frames it takes
 * (the rest go to k_pack by list).
 * ==================================================================================== */

__device__ __forceinline__ bool packw_frame_ok(const FrameArgs& a, int64_t f) {
    for (int c = 0; c < a.channels; ++c) {
        const int64_t u = f * a.channels + c;
        if ((unit_len(a, u) >> a.meta[u].part_order) < 8) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t crc_fold_word(uint32_t c, uint32_t w, const uint16_t* ct) {
    return (uint32_t)ct[3 * 256 + ((c >> 8) ^ (w >> 24))] ^ (uint32_t)ct[2 * 256 + ((c ^ (w >> 16)) & 0xFF)] ^
           (uint32_t)ct[256 + ((w >> 8) & 0xFF)] ^ (uint32_t)ct[w & 0xFF];
}

template <int MAXC, int NT, int RW> /* NT: the launch's threads; RW: ring words */
__device__ __forceinline__ void packw_frame(const FrameArgs& a) {
    constexpr uint32_t RM = RW - 1;
    constexpr int CH = 2 * NT;                    /* words leaving the ring together */
    constexpr int CHL = NT == 64 ? 9 : NT == 128 ? 10 : 11; /* x^(8 * 4 CH) = x^(8 * 2^CHL) */
    static_assert(NT == 64 || NT == 128 || NT == 256, "k_packw runs 64, 128 or 256 threads");
    __shared__ __align__(16) uint32_t win[RW];
    __shared__ __align__(16) uint16_t ct[4 * 256];
    __shared__ __align__(16) uint16_t pwc[512]; /* c -> c * x^(8 * CH * 4) */
    __shared__ uint8_t hdr[16];
    __shared__ uint32_t sub_start[9];
    __shared__ int32_t cnt14[8];
    __shared__ uint32_t red[NT / 64];
    __shared__ uint32_t red2[NT / 64];
    __shared__ int hb_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t f = blockIdx.x;
    if (a.offsets[a.n_frames] > a.capacity) return; /* k_pack reports it */
    if (a.status[f] != 0) return;
    if (!packw_frame_ok(a, f)) { /* k_pack writes it */
        if (tid == 0) a.slow_list[atomicAdd(a.slow_count, 1ull)] = f;
        return;
    }
    const int64_t F = a.offsets[f], Fend = a.offsets[f + 1];
    const int64_t lead = (int64_t)(((uintptr_t)a.out + (uintptr_t)F) & 15);
    const int64_t Fa = F - lead;            /* output byte of window bit 0 (16-byte aligned) */
    const uint32_t A = (uint32_t)(8 * lead); /* window bit of the frame's first bit */
    const int64_t u0 = f * a.channels;
    const int C = a.channels;
    const uint16_t* __restrict__ pw = a.crc_pow;
    for (int i = tid; i < 128; i += NT) reinterpret_cast<uint4*>(ct)[i] = reinterpret_cast<const uint4*>(a.crc_slice)[i];
    for (int i = tid; i < 64; i += NT)
        reinterpret_cast<uint4*>(pwc)[i] = reinterpret_cast<const uint4*>(pw + CHL * 512)[i];
    for (int i = tid; i < RW / 4; i += NT) reinterpret_cast<uint4*>(win)[i] = uint4{0, 0, 0, 0};
    if (tid < 8) cnt14[tid] = 0;
    if (tid == 0) hb_s = frame_header(a.first_frame + f, unit_len(a, u0), hdr);
    __syncthreads();
    for (int c = 0; c < C; ++c) {
        const flacmi_unit_meta& m = a.meta[u0 + c];
        if (m.coding_method == 5) {
            const int32_t* rp = a.rice_params + (u0 + c) * a.params_stride;
            int cnt = 0;
            for (int k = tid; k < m.n_parts; k += NT) cnt += rp[k] > 14 ? 1 : 0;
            if (cnt) atomicAdd(&cnt14[c], cnt);
        }
    }
    __syncthreads();
    const int hb = hb_s;
    if (tid == 0) {
        uint32_t s = A + 8u * (uint32_t)hb;
        for (int c = 0; c < C; ++c) {
            const flacmi_unit_meta& m = a.meta[u0 + c];
            sub_start[c] = s;
            s += sub_prefix_bits(m, a.sample_size, a.q) + (uint32_t)sub_residual_bits(m, cnt14[c]);
        }
        sub_start[C] = s;
    }
    __syncthreads();

    uint32_t fl = 0;    /* ring words below fl have left (uniform) */
    uint32_t crc_t = 0; /* this thread's running CRC over its words of the chunks that left */
    /* the w-bit field val (1 <= w <= 32) at window bit P: one or two ORs, words outside the
     * ring's span skipped */
    auto ring_or = [&](uint32_t P, uint32_t val, uint32_t w) __attribute__((always_inline)) {
        const uint64_t t = (uint64_t)val << (64u - (P & 31u) - w);
        const uint32_t wi = P >> 5;
        if (wi - fl < (uint32_t)RW) atomicOr(&win[wi & RM], (uint32_t)(t >> 32));
        if (wi + 1u - fl < (uint32_t)RW) atomicOr(&win[(wi + 1u) & RM], (uint32_t)t);
    };
    /* whole chunks below ring word upto leave: CRC share, store, zero; frame bytes are
     * [fb0, fb1) in window bytes */
    const uint32_t fb0 = (uint32_t)lead, fb1 = (uint32_t)(lead + (Fend - F));
    uint8_t* __restrict__ ob = a.out + Fa; /* output byte of window byte 0 (never written below F) */
    auto store8 = [&](uint32_t rb, uint2 w) __attribute__((always_inline)) {
        if (rb >= fb0 && rb + 8u <= fb1) {
            *reinterpret_cast<uint2*>(ob + rb) = uint2{__builtin_bswap32(w.x), __builtin_bswap32(w.y)};
        } else {
#pragma unroll 1
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t wj = j < 4 ? w.x : w.y;
                if (rb + j >= fb0 && rb + j < fb1) ob[rb + j] = (uint8_t)(wj >> (24 - 8 * (j & 3)));
            }
        }
    };
    auto leave = [&](uint32_t upto) __attribute__((always_inline)) {
        if (upto - fl < (uint32_t)CH) return;
        do {
            const uint32_t k = fl + 2u * (uint32_t)tid;
            uint2* wp = reinterpret_cast<uint2*>(&win[k & RM]);
            const uint2 w = *wp;
            *wp = uint2{0, 0};
            const uint32_t c = crc_fold_word(crc_fold_word(0, w.x, ct), w.y, ct);
            crc_t = ((uint32_t)pwc[crc_t & 0xFF] ^ (uint32_t)pwc[256 + (crc_t >> 8)]) ^ c;
            store8(4u * k, w);
            fl += (uint32_t)CH;
        } while (upto - fl >= (uint32_t)CH);
        __syncthreads(); /* zeroed words are written again by the next segment */
    };

    /* the frame header and a subframe's header fields (< 1600 bits) always fit the ring
     * above the < CH words still waiting */
    if (tid < hb) ring_or(A + 8u * tid, hdr[tid], 8);
    __syncthreads();
    leave((A + 8u * hb) >> 5);
    const int ss = a.sample_size, q = a.q;
    for (int c = 0; c < C; ++c) {
        const int64_t u = u0 + c;
        const flacmi_unit_meta& m = a.meta[u];
        const int n = unit_len(a, u);
        const int order = m.order, ncoefs = m.ncoefs, method = m.coding_method;
        const bool lpc = m.kind == FLACMI_KIND_LPC;
        const uint32_t s0 = sub_start[c];
        const uint32_t pre = sub_prefix_bits(m, ss, q);
        const int nfields = 1 + order + (lpc ? 2 + ncoefs : 0) + 2;
        {
            for (int t = tid; t < nfields; t += NT) {
                uint32_t pos, v, w;
                const uint32_t b = s0 + 8 + (uint32_t)order * ss;
                const int t2 = t - 1 - order;
                if (t == 0) {
                    pos = s0;
                    v = lpc ? (uint32_t)((0x20 | (order - 1)) << 1) : (uint32_t)((0x08 | order) << 1);
                    w = 8;
                } else if (t <= order) {
                    const int j = t - 1;
                    const int32_t x = a.sample_bytes == 2 ? (int32_t)((const int16_t*)a.samples)[u * a.stride + j]
                                                          : ((const int32_t*)a.samples)[u * a.stride + j];
                    pos = s0 + 8 + (uint32_t)j * ss;
                    v = (uint32_t)x & (ss == 32 ? ~0u : ((1u << ss) - 1u));
                    w = (uint32_t)ss;
                } else if (lpc && t2 == 0) {
                    pos = b;
                    v = (uint32_t)((q - 1) & 15);
                    w = 4;
                } else if (lpc && t2 == 1) {
                    pos = b + 4;
                    v = (uint32_t)(m.shift & 31);
                    w = 5;
                } else if (lpc && t2 < 2 + ncoefs) {
                    const int j = t2 - 2;
                    pos = b + 9 + (uint32_t)j * q;
                    v = (uint32_t)m.coefs[j] & ((1u << q) - 1u);
                    w = (uint32_t)q;
                } else {
                    const int t3 = t2 - (lpc ? 2 + ncoefs : 0);
                    const uint32_t b2 = b + (lpc ? 9u + (uint32_t)ncoefs * q : 0u);
                    pos = t3 == 0 ? b2 : b2 + 2;
                    v = t3 == 0 ? (method == 5 ? 1u : 0u) : (uint32_t)(m.part_order & 15);
                    w = t3 == 0 ? 2u : 4u;
                }
                ring_or(pos, v, w);
            }
        }
        __syncthreads();
        leave((s0 + pre) >> 5);
        /* residual: tiles of NT * MAXC chunks, thread t's run [k0, k1) of each */
        const int ps = n >> m.part_order;
        const int32_t* __restrict__ rp = a.rice_params + u * a.params_stride;
        const uint32_t* __restrict__ zrow = reinterpret_cast<const uint32_t*>(a.residual) + u * a.residual_stride;
        const int nch = (n + 7) >> 3;
        const uint32_t pmask_m = (1u << method) - 1u;
        uint32_t tile_base = s0 + pre;
        for (int tb = 0; tb < nch; tb += NT * MAXC) {
            const int k0 = tb + tid * MAXC, k1 = min(k0 + MAXC, nch);
            uint32_t z[MAXC][8];
            int pa[MAXC], pb[MAXC], bnd[MAXC], pt0[MAXC];
            uint32_t tsum = 0;
#pragma unroll
            for (int j = 0; j < MAXC; ++j) {
                const int k = k0 + j;
                const int i0 = 8 * k;
                pa[j] = pb[j] = 0;
                bnd[j] = 1 << 30;
                pt0[j] = 0;
                if (k < k1) {
                    if (i0 + 8 <= n) {
                        const uint4 v0 = *reinterpret_cast<const uint4*>(zrow + i0);
                        const uint4 v1 = *reinterpret_cast<const uint4*>(zrow + i0 + 4);
                        z[j][0] = v0.x; z[j][1] = v0.y; z[j][2] = v0.z; z[j][3] = v0.w;
                        z[j][4] = v1.x; z[j][5] = v1.y; z[j][6] = v1.z; z[j][7] = v1.w;
                    } else { /* the row's last chunk: no reads past its end */
#pragma unroll
                        for (int e = 0; e < 8; ++e) z[j][e] = i0 + e < n ? zrow[i0 + e] : 0u;
                    }
                    const int part0 = i0 / ps;
                    pt0[j] = part0;
                    const int b1 = (part0 + 1) * ps;
                    pa[j] = rp[part0];
                    pb[j] = (b1 < n && b1 <= i0 + 7) ? rp[part0 + 1] : pa[j];
                    bnd[j] = b1;
                    if (i0 > order && i0 + 8 <= n && b1 >= i0 + 8) {
                        const int p = pa[j];
                        uint32_t qs = 0;
#pragma unroll
                        for (int e = 0; e < 8; ++e) qs += z[j][e] >> p;
                        tsum += qs + 8u * (uint32_t)(p + 1) + (i0 == part0 * ps ? (uint32_t)method : 0u);
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const int i = i0 + e;
                            const int p = i >= b1 ? pb[j] : pa[j];
                            const bool valid = i >= order && i < n;
                            const bool first = i == order || (i > order && (i == b1 || i == part0 * ps));
                            tsum += valid ? (first ? (uint32_t)method : 0u) + (z[j][e] >> p) + 1u + (uint32_t)p : 0u;
                        }
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) z[j][e] = 0;
                }
            }
            /* workgroup exclusive scan of tsum */
            uint32_t v = tsum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += t;
            }
            if (lane == 63) red[wid] = v;
            __syncthreads();
            uint32_t pre_w = 0, tot = 0;
#pragma unroll
            for (int w2 = 0; w2 < NT / 64; ++w2) {
                const uint32_t s = red[w2];
                pre_w += w2 < wid ? s : 0u;
                tot += s;
            }
            const uint32_t tstart = tile_base + pre_w + v - tsum;
            const uint32_t te = tile_base + tot;
            /* a tile that overruns the ring writes what fits, the full ring leaves, and it
             * runs again */
            bool again;
            do {
                uint32_t pos = tstart;
                asm volatile("" : "+v"(pos)); /* opaque: nothing of the body is hoisted out of the redo loop */
#pragma unroll
                for (int j = 0; j < MAXC; ++j) {
                    const int k = k0 + j;
                    if (k < k1) {
                        const int i0 = 8 * k;
                        const int part0 = pt0[j];
                        if (i0 > order && i0 + 8 <= n && bnd[j] >= i0 + 8) {
                            const int p = pa[j];
                            if (i0 == part0 * ps) {
                                ring_or(pos, (uint32_t)p & pmask_m, (uint32_t)method);
                                pos += (uint32_t)method;
                            }
                            const uint32_t one = 1u << p, wc = (uint32_t)p + 1u;
#pragma unroll
                            for (int e = 0; e < 8; ++e) {
                                uint32_t zk = z[j][e];
                                /* opaque per value: the 8 codes are formed one after the other,
                                 * not all up front (about 45 fewer VGPRs for 2 chunks) */
                                asm volatile("" : "+v"(zk));
                                const uint32_t P = pos + (zk >> p);
                                ring_or(P, one | (zk & (one - 1u)), wc);
                                pos = P + wc;
                            }
                        } else { /* the warm-up's chunk, the unit's end, a partition boundary inside */
#pragma unroll 1
                            for (int e = 0; e < 8; ++e) {
                                uint32_t zk = z[j][0];
#pragma unroll
                                for (int e2 = 1; e2 < 8; ++e2) zk = e == e2 ? z[j][e2] : zk;
                                const int i = i0 + e;
                                if (i >= order && i < n) {
                                    const int p = i >= bnd[j] ? pb[j] : pa[j];
                                    if (i == order || i == bnd[j] || i == part0 * ps) {
                                        ring_or(pos, (uint32_t)p & pmask_m, (uint32_t)method);
                                        pos += (uint32_t)method;
                                    }
                                    const uint32_t P = pos + (zk >> p);
                                    ring_or(P, (1u << p) | (zk & ((1u << p) - 1u)), (uint32_t)p + 1u); /* p <= 30 */
                                    pos = P + (uint32_t)p + 1u;
                                }
                            }
                        }
                    }
                }
                __syncthreads();
                again = ((te - 1u) >> 5) - fl >= (uint32_t)RW;
                leave(again ? fl + (uint32_t)RW : te >> 5);
            } while (again);
            tile_base = te;
        }
    }

    /* CRC-16 of bytes [F, E), E = Fend - 2: the chunks that left (the running CRCs, thread
     * t's 8-byte words before thread t + 1's in every chunk, joined by a lane tree at
     * x^(8 * 8 * 2^l) and the waves at x^(8 * 512)), then the ring's words below E (k_pack32's
     * end fold from word fl), the first shifted past the second */
    const int64_t E = Fend - 2;
    {
        const int nfull = (int)(((E - Fa) >> 2) - (int64_t)fl);
        int ls = 0;
        while ((NT << ls) < nfull) ++ls;
        const int spw = 1 << ls;
        const int w1 = nfull - (NT - 1 - tid) * spw, w0 = w1 - spw;
        auto mulx = [&](uint32_t c, int bl) __attribute__((always_inline)) {
            return (uint32_t)pw[bl * 512 + (c & 0xFF)] ^ (uint32_t)pw[bl * 512 + 256 + (c >> 8)];
        };
        uint32_t crc = 0;
        for (int k = max(w0, 0); k < w1; ++k) crc = crc_fold_word(crc, win[(fl + (uint32_t)k) & RM], ct);
        uint32_t x = crc_t;
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            const bool right = (lane >> l) & 1;
            const uint32_t oc = (uint32_t)__shfl_xor((int)crc, 1 << l);
            crc = mulx(right ? oc : crc, ls + 2 + l) ^ (right ? crc : oc);
            const uint32_t ox = (uint32_t)__shfl_xor((int)x, 1 << l);
            x = mulx(right ? ox : x, 3 + l) ^ (right ? x : ox);
        }
        if (lane == 0) {
            red[wid] = crc;
            red2[wid] = x;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t tcrc = 0, xc = 0;
            for (int w2 = 0; w2 < NT / 64; ++w2) {
                tcrc = (w2 ? mulx(tcrc, ls + 8) : 0u) ^ red[w2];
                xc = (w2 ? mulx(xc, 9) : 0u) ^ red2[w2];
            }
            const int tail = (int)(E - Fa - 4 * (int64_t)fl) - 4 * nfull;
            const uint32_t tw = win[(fl + (uint32_t)nfull) & RM];
            for (int j = 0; j < tail; ++j) tcrc = ((tcrc << 8) & 0xFFFF) ^ (uint32_t)ct[(tcrc >> 8) ^ ((tw >> (24 - 8 * j)) & 0xFF)];
            const uint32_t all = crc16_mulpow(xc, E - Fa - 4 * (int64_t)fl, pw) ^ tcrc;
            ring_or((uint32_t)(8 * (E - Fa)), all & 0xFFFF, 16);
        }
        __syncthreads();
    }
    /* the ring's last words */
    const uint32_t endw = (uint32_t)((Fend - Fa + 3) >> 2);
    for (uint32_t k = fl + 2u * (uint32_t)tid; k < endw; k += 2u * NT) {
        store8(4u * k, *reinterpret_cast<const uint2*>(&win[k & RM]));
    }
}

/* the default build: 64 threads (one wave: the workgroup's barriers are one wave's), a 4 KB
 * ring, one chunk a thread, held to 6 waves a SIMD (76 VGPRs, no spills).  c3 frames, same
 * box: 256 threads on a 16 KB ring 5.53-5.56 ms, 128 threads on 8 KB 5.13-5.14, 64 on 4 KB
 * 5.08.  k_packw_redo_test's MAXC = 4 (knob 3) gives 2048-value tiles, about 1400 ring words for 24-bit frames,
 * for the tests of the redo of a tile that overruns the ring. */
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_packw(FrameArgs a) {
    packw_frame<1, 64, 1024>(a);
}
__global__ __launch_bounds__(64) void k_packw_redo_test(FrameArgs a) { /* knob 3 (no occupancy floor) */
    packw_frame<4, 64, 1024>(a);
}
/* A/B builds: 256 threads on a 16 KB ring (the first default), 128 threads on an 8 KB ring */
__global__ __launch_bounds__(kPackThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_packw256(FrameArgs a) {
    packw_frame<1, kPackThreads, kWinWords>(a);
}
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_packw128(FrameArgs a) {
    packw_frame<1, 128, 2048>(a);
}
/* samples of <= 16 bits: a 2 KB ring (5.2 KB of LDS: 24 workgroups a CU, the VGPR limit,
 * instead of 21).  A 512-value tile fits it above the < 128 waiting words up to 24 bits a
 * value; 16-bit residuals stay far below.  c2 frames 8.01 -> 7.35 ms same box (c3's 24-bit
 * frames only 5.02 -> 4.93, with tiles near the limit: they keep the 4 KB ring). */
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_packw2k(FrameArgs a) {
    packw_frame<1, 64, 512>(a);
}

hipError_t launch_frame_sizes(const FrameArgs& a, int64_t* bsum, hipStream_t s) {
    if (a.n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_frame_sizes, dim3((unsigned)((a.n_frames + 3) / 4)), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t n = a.n_frames;
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nb), dim3(256), 0, s, a.offsets + 1, n, bsum);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, s, bsum, nb);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(256), 0, s, a.offsets + 1, n, (const int64_t*)bsum);
    return hipGetLastError();
}

int64_t frame_scan_blocks(int64_t n_frames) { return (n_frames + kScanBlock - 1) / kScanBlock; }

hipError_t launch_pack(const FrameArgs& a, hipStream_t s) {
    if (a.n_frames <= 0) return hipSuccess;
    /* workgroup: 8-value chunks in as few full tiles of <= 256 threads as possible */
    const int nch = (a.block_len + 7) / 8;
    const int tiles = (nch + kPackThreads - 1) / kPackThreads;
    int nt = 64 * ((nch + 64 * tiles - 1) / (64 * tiles));
    nt = nt < 64 ? 64 : nt;
    if (a.residual_bytes == 8) {
        hipLaunchKernelGGL(k_pack<uint64_t>, dim3((unsigned)a.n_frames), dim3(nt), 0, s, a);
        return hipGetLastError();
    }
    FrameArgs b = a;
    /* knob FLACMI_PACK_GENERIC: 1 every frame through k_pack; 2 no k_packw (k_pack32 for the
     * frames it fits, k_pack for the rest: the writer before k_packw); 3 k_packw with
     * 2048-value tiles (tiles that overrun the ring: the test of its redo path); 6 / 8 k_packw
     * built for 256 / 128 threads (A/B); 7 as 2 with k_pack32 on its 16 KB window only.
     * Default: k_packw for every batch of 32-bit residual rows it can read with 16-byte loads
     * (one wave a frame beat k_pack32's one workgroup a frame on config 2 too: 8.02 against
     * 8.48-8.49 ms per 1e6 frames, same box) */
    const int pack_generic = knob(kKnobPackGeneric);
    const bool no_pack32 = pack_generic == 1;
    const bool no_packw = pack_generic == 1 || pack_generic == 2 || pack_generic == 7;
    /* the ablation switch, read once per process (no getenv per launch) */
    static const int ablate = [] {
        const char* e = getenv("FLACMI_PACK_ABLATE");
        return e ? atoi(e) : 0;
    }();
    /* k_pack32 / k_packw read residual rows with 16-byte loads */
    const bool vec_ok = ((uintptr_t)a.residual & 15) == 0 && (a.residual_stride & 3) == 0;
    const bool wide = !(tiles == 1 || (nch + nt - 1) / nt <= kMaxC);
    b.ablate = ablate;
    if (vec_ok && !no_packw) {
        /* k_packw, 64 threads, 1 chunk a thread a tile (a tile of 512 values fits the ring
         * above the < 128 words still waiting to leave up to 56 bits a value on average; a
         * longer one, e.g. long unary runs of outliers, takes the redo path) */
        b.pack_split = 1;
        hipError_t e0 = hipMemsetAsync(b.slow_count, 0, sizeof(unsigned long long), s);
        if (e0 != hipSuccess) return e0;
        const dim3 g((unsigned)a.n_frames);
        if (pack_generic == 3) hipLaunchKernelGGL(k_packw_redo_test, g, dim3(64), 0, s, b);
        else if (pack_generic == 6) hipLaunchKernelGGL(k_packw256, g, dim3(kPackThreads), 0, s, b);
        else if (pack_generic == 8) hipLaunchKernelGGL(k_packw128, g, dim3(128), 0, s, b);
        else if (a.sample_size <= 16) hipLaunchKernelGGL(k_packw2k, g, dim3(64), 0, s, b);
        else hipLaunchKernelGGL(k_packw, g, dim3(64), 0, s, b);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const int64_t grid = a.n_frames < 4096 ? a.n_frames : 4096;
        hipLaunchKernelGGL(k_pack<uint32_t>, dim3((unsigned)grid), dim3(nt), 0, s, b);
        return hipGetLastError();
    }
    b.pack_split = !wide && vec_ok && !no_pack32;
    if (b.pack_split) {
        hipError_t e0 = hipMemsetAsync(b.slow_count, 0, sizeof(unsigned long long), s);
        if (e0 != hipSuccess) return e0;
        const int cpt = (nch + nt - 1) / nt;
        const dim3 g((unsigned)a.n_frames), t(nt);
        /* the small window when a verbatim frame fits it with room (Rice frames larger than
         * that go to k_pack) */
        const int64_t verb = (int64_t)a.block_len * a.sample_size * a.channels / 8 + 64;
        const bool small = verb + verb / 4 <= 4LL * kWinSmall && pack_generic != 7;
        if (small) {
            if (cpt <= 2) hipLaunchKernelGGL((k_pack32<2, kWinSmall, 7>), g, t, 0, s, b);
            else if (cpt == 3) hipLaunchKernelGGL((k_pack32<3, kWinSmall, 7>), g, t, 0, s, b);
            else hipLaunchKernelGGL((k_pack32<kMaxC, kWinSmall, 5>), g, t, 0, s, b);
        } else {
            if (cpt <= 2) hipLaunchKernelGGL((k_pack32<2, kWinWords, 1>), g, t, 0, s, b);
            else if (cpt == 3) hipLaunchKernelGGL((k_pack32<3, kWinWords, 1>), g, t, 0, s, b);
            else hipLaunchKernelGGL((k_pack32<kMaxC, kWinWords, 1>), g, t, 0, s, b);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const int64_t grid = b.pack_split ? (a.n_frames < 4096 ? a.n_frames : 4096) : a.n_frames;
    hipLaunchKernelGGL(k_pack<uint32_t>, dim3((unsigned)grid), dim3(nt), 0, s, b);
    return hipGetLastError();
}

}  // namespace flacmi
