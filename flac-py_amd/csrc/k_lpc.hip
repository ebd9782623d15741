/* k_lpc.hip — autocorrelation + Levinson-Durbin + quantisation, one lane per unit
 * (see device_common.h for the design notes). */
#include <type_traits>

#include <map>
#include <mutex>
#include <utility>

#include "device_common.h"

namespace flacmi {

/* ====================================================================================
 * k_lpc: autocorrelation + Levinson-Durbin + quantisation, one lane per unit
 * ==================================================================================== */

template <int LMAX>
__device__ __forceinline__ void write_quant(int32_t* rec, int L, int p, const int32_t* q, int nq,
                                            int shift) {
    rec[2 + p - 1] = shift;
    int32_t* c = rec + 2 + L + (p * (p - 1)) / 2;
#pragma unroll
    for (int j = 0; j < LMAX; ++j)
        if (j < p) c[j] = j < nq ? q[j] : 0;
}

/* Levinson-Durbin at max order with a snapshot per order (encoder.py:453-479), each
 * snapshot quantised (encoder.py:482-534), into the unit's LPC record */
template <int LMAX>
__device__ __forceinline__ void lpc_finish(const double (&acc)[LMAX + 1], const LpcArgs& a, int32_t* __restrict__ rec) {
    const int L = a.L, q = a.q;
    const pym::PowTables PT{c_log_hdr, c_log_tab, c_exp_hdr, c_exp_tab};
    double c[LMAX + 1];
    c[0] = 1.0;
#pragma unroll
    for (int j = 1; j <= LMAX; ++j) c[j] = 0.0;
    double err = acc[0];
    int lst = ST_OK, lsite = 0, qst = ST_OK, qsite = 0;
    uint32_t negmask = 0;
    const double qmax = (double)((1LL << (q - 1)) - 1);
    const double qmin = -(double)(1LL << (q - 1));
    static_for<LMAX>([&](auto K_) {
        constexpr int k = K_;
        if (k < L && lst == ST_OK) {
            double lam = 0.0;
#pragma unroll
            for (int j = 0; j <= k; ++j) lam = lam - c[j] * acc[k + 1 - j];
            if (err == 0.0) {
                lst = ST_ZERODIV;
                lsite = FLACMI_SITE_LEVINSON_DIV;
            } else {
                lam = lam / err;
#pragma unroll
                for (int nn = 0; nn <= (k + 1) / 2; ++nn) {
                    const double tmp = c[k + 1 - nn] + lam * c[nn];
                    c[nn] = c[nn] + lam * c[k + 1 - nn];
                    c[k + 1 - nn] = tmp;
                }
                int pst;
                const double l2 = pym::py_pow2(lam, PT, &pst);
                if (pst) {
                    lst = ST_OVERFLOW;
                    lsite = FLACMI_SITE_LEVINSON_POW;
                } else {
                    err = err * (1.0 - l2);
                }
            }
            /* quantise order p = k + 1 (encoder.py:482-534) unless an earlier order failed */
            if (lst == ST_OK && qst == ST_OK) {
                const int p = k + 1;
                double cm = __builtin_fabs(c[1]);
#pragma unroll
                for (int j = 2; j <= LMAX; ++j)
                    if (j <= p && __builtin_fabs(c[j]) > cm) cm = __builtin_fabs(c[j]);
                /* the quantised coefficients go straight into the record (no qv[LMAX] array held
                 * beside c[] and acc[]: 32 VGPRs at L = 32); an order that fails leaves the
                 * record's status set, so what it wrote is never read */
                int32_t* __restrict__ cq = rec + 2 + L + (p * (p - 1)) / 2;
                int shift = 0;
                if (!(cm > 0.0)) {
                    qst = ST_ASSERT;
                    qsite = FLACMI_SITE_QUANT_CMAX;
                } else if (__builtin_isinf(cm)) {
                    qst = ST_OVERFLOW;
                    qsite = FLACMI_SITE_QUANT_LOG2;
                } else {
                    shift = q - pym::py_floor_log2(cm, a.log2thr) - 2;
                    if (shift > 15) shift = 15;
                    if (shift < -16) {
                        qst = ST_ASSERT;
                        qsite = FLACMI_SITE_QUANT_SHIFT;
                    } else {
                        const bool neg = shift < 0;
                        const double scale = pow2_exact(neg ? -shift : shift);
                        double e = 0.0;
#pragma unroll
                        for (int j = 1; j <= LMAX; ++j) {
                            if (j <= p && qst == ST_OK) {
                                e = e + c[j] * scale;
                                if (__builtin_isinf(e)) {
                                    qst = ST_OVERFLOW;
                                    qsite = FLACMI_SITE_QUANT_ROUND_INF;
                                } else if (__builtin_isnan(e)) {
                                    qst = ST_VALUE;
                                    qsite = FLACMI_SITE_QUANT_ROUND_NAN;
                                } else {
                                    const double r = __builtin_rint(e);
                                    const double qq = r < qmin ? qmin : (r > qmax ? qmax : r);
                                    e = e - qq;
                                    cq[j - 1] = (int32_t)qq;
                                }
                            }
                        }
                        if (qst == ST_OK) {
                            if (neg) { /* ([], 0) (encoder.py:523-532): no coefficients, shift 0 */
                                negmask |= 1u << k;
                                shift = 0;
#pragma unroll
                                for (int j = 0; j < LMAX; ++j)
                                    if (j < p) cq[j] = 0;
                            }
                            rec[2 + p - 1] = shift;
                        }
                    }
                }
            }
        }
    });
    int st = lst != ST_OK ? lst : qst;
    int site = lst != ST_OK ? lsite : qsite;
    if (st == ST_OK && L == 0) { /* min() over no candidates (encoder.py:404) */
        st = ST_VALUE;
        site = FLACMI_SITE_LPC_EMPTY;
    }
    rec[0] = st | (site << 16);
    rec[1] = (int32_t)negmask;
}

/* ACF_IN: the autocorrelation is read from a.acf ([count][33]) instead of computed from
 * samples -- the entry point flacmi_device_lpc_from_acf uses to drive Levinson-Durbin and
 * the quantiser into the overflow sites integer PCM never reaches. */
/* three waves per SIMD for the common orders (L <= 12: <= 168 VGPRs); two for 32-bit samples
 * at L = 32 (208 VGPRs: the ring cycles of the two tapers and of the rectangle run as three
 * loops, one path each; with one loop holding both paths the allocator needed > 256) */
constexpr int lpc_waves(int lmax, int sample_bytes = 4) { return lmax <= 12 ? 3 : sample_bytes == 4 ? 2 : 1; }

template <int LMAX, typename SampleT, bool ACF_IN = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(lpc_waves(LMAX, (int)sizeof(SampleT))))) void k_lpc(LpcArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.count) return;
    const int64_t u = a.unit0 + gid;
    const SampleT* __restrict__ x = (const SampleT*)a.samples + u * a.stride;
    int32_t* __restrict__ rec = a.rec + gid * a.rec_words;
    const int n = a.n, L = a.L;

    constexpr int S = ((LMAX + 1 + 7) / 8) * 8;
    double acc[LMAX + 1];
    if constexpr (ACF_IN) {
#pragma unroll
        for (int l = 0; l <= LMAX; ++l) acc[l] = l <= L ? a.acf[gid * 33 + l] : 0.0;
    } else {
    if (n >= 4 && n <= 7) { /* tukey: nr == 0 -> pi * 0 / 0 (encoder.py:437) */
        rec[0] = ST_ZERODIV | (FLACMI_SITE_TUKEY << 16);
        rec[1] = 0;
        if (a.acf)
            for (int l = 0; l < 33; ++l) a.acf[gid * 33 + l] = 0.0;
        return;
    }

    /* ---- autocorrelation: acc[l] = sum_{m} a[m-l] * a[m], m = 0 .. n-2 ---- */
    double ring[S];
#pragma unroll
    for (int t = 0; t < S; ++t) ring[t] = 0.0;
#pragma unroll
    for (int l = 0; l <= LMAX; ++l) acc[l] = 0.0;
    const int M = n - 1; /* the last sample never enters a product (encoder.py:449) */
    /* the window through the constant address space: scalar loads (a global pointer gets
     * per-lane vector loads, each waited for with vmcnt(0) -- which also waits for the
     * samples prefetched a cycle ahead) */
    const __attribute__((address_space(4))) double* win = (const __attribute__((address_space(4))) double*)a.window;
    /* Samples arrive in load blocks of SB per lane (64 B: a whole half cache line per row
     * per visit), kept packed (int16 pairs) and prefetched one block ahead; each block is
     * processed as SB / S ring-aligned sub-blocks of S samples. */
    constexpr int PK = sizeof(SampleT) == 2 ? 2 : 1; /* samples per 32-bit word */
    constexpr int SB = sizeof(SampleT) == 2 ? 2 * S : S;
    constexpr int W = SB / PK;
    const int nblk = (M + SB - 1) / SB;
    uint32_t cur[W];
    auto load = [&](int m0, uint32_t (&v)[W]) __attribute__((always_inline)) {
        if (m0 + SB <= M) {
#pragma unroll
            for (int g = 0; g < W / 4; ++g) {
                const uint4 q = *reinterpret_cast<const uint4*>(x + m0 + 4 * PK * g);
                v[4 * g] = q.x;
                v[4 * g + 1] = q.y;
                v[4 * g + 2] = q.z;
                v[4 * g + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if constexpr (PK == 2) {
                    const uint32_t lo = (m0 + 2 * w < M) ? (uint16_t)x[m0 + 2 * w] : 0u;
                    const uint32_t hi = (m0 + 2 * w + 1 < M) ? (uint16_t)x[m0 + 2 * w + 1] : 0u;
                    v[w] = lo | (hi << 16);
                } else {
                    v[w] = (m0 + w < M) ? (uint32_t)x[m0 + w] : 0u;
                }
            }
        }
    };
    auto sample = [&](const uint32_t (&v)[W], int t) __attribute__((always_inline)) -> int32_t {
        if constexpr (PK == 2) return (t & 1) ? (int32_t)v[t >> 1] >> 16 : (int32_t)(v[t >> 1] << 16) >> 16;
        return (int32_t)v[t];
    };
    if constexpr (PK == 1) {
        /* 32-bit samples (L up to 32, S = 40): loading whole S-sample blocks would hold 2 x 40
         * sample registers beside the 33 accumulators and the 40-slot ring (one wave per SIMD,
         * accumulators spilled to AGPRs).  Instead groups of G samples are prefetched one ring
         * cycle ahead while the ring cycles through its S slots (static indices throughout). */
        constexpr int G = 8;
        static_assert(S % G == 0, "ring length a multiple of the load group");
        const int ncyc = (M + S - 1) / S;
        /* FULL: the group lies inside [0, M) (the caller knows; no branch, so the waits the
         * compiler places before each use count only the loads issued since) */
        auto loadg = [&](int m0, uint32_t (&v)[G], auto fullc) __attribute__((always_inline)) {
            if (decltype(fullc)::value || m0 + G <= M) {
                const uint4 q0 = *reinterpret_cast<const uint4*>(x + m0);
                const uint4 q1 = *reinterpret_cast<const uint4*>(x + m0 + 4);
                v[0] = q0.x; v[1] = q0.y; v[2] = q0.z; v[3] = q0.w;
                v[4] = q1.x; v[5] = q1.y; v[6] = q1.z; v[7] = q1.w;
            } else {
#pragma unroll
                for (int k = 0; k < G; ++k) v[k] = (m0 + k < M) ? (uint32_t)x[m0 + k] : 0u;
            }
        };
        using T0 = std::integral_constant<bool, false>;
        using T1 = std::integral_constant<bool, true>;
        /* the samples of one whole ring cycle in flight: group g of cycle c + 1 is loaded into
         * gb[g] as soon as cycle c has used it (an HBM round trip is longer than one group's
         * 8 x 33 f64 operations at two waves per SIMD) */
        uint32_t gb[S / G][G];
#pragma unroll
        for (int g = 0; g < S / G; ++g) loadg(g * G, gb[g], T0{});
        __builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0): the loops below enter with nothing in flight */
        /* one ring cycle (S samples); RECT: inside the window's rectangle (see below); FULL:
         * the next cycle lies inside [0, M) */
        auto cycle = [&](int c, auto rectc, auto fullc) __attribute__((always_inline)) {
            constexpr bool RECT = decltype(rectc)::value;
            const int m0 = c * S;
#pragma unroll
            for (int g = 0; g < S / G; ++g) {
                const int mg = m0 + g * G;
                if constexpr (RECT) { /* exact integer products: one fused op per term (see below) */
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int t = g * G + k;
                        const double av = (double)(int32_t)gb[g][k];
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) acc[l] = __builtin_fma(ring[(t - l + S) % S], av, acc[l]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int t = g * G + k;
                        const double av = (double)(int32_t)gb[g][k] * win[mg + k];
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) {
                            const double prev = ring[(t - l + S) % S];
                            acc[l] = acc[l] + prev * av;
                        }
                    }
                }
                /* pinned here: left to itself the scheduler sinks the loads to the end of the
                 * cycle, and the next cycle then waits on them at once */
                __builtin_amdgcn_sched_barrier(0);
                loadg(mg + S, gb[g], fullc);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        /* Cycles c < cf prefetch a whole cycle inside [0, M).  Among them the rectangle's cycles
         * form one run [c1, c2); the taper cycles before and after it share one loop (one copy
         * of the code); the last cycles (c >= cf) take the multiply-and-add path, which is the
         * reference's own arithmetic and so exact inside the rectangle too. */
        const int cf = M / S - 1 > 0 ? M / S - 1 : 0;
        int c1 = (a.fuse_lo + LMAX + S - 1) / S;
        if (a.fuse_lo + LMAX <= 0) c1 = 0;
        int c2 = a.fuse_hi / S; /* c * S + S <= fuse_hi  <=>  c < fuse_hi / S */
        if (c2 > cf) c2 = cf;
        if (c1 > c2) c1 = c2;
        const int ntap = c1 + (cf - c2);
        for (int i = 0; i < c1; ++i) cycle(i, T0{}, T1{});
        for (int c = c1; c < c2; ++c) cycle(c, T1{}, T1{});
        for (int c = c2; c < cf; ++c) cycle(c, T0{}, T1{});
        (void)ntap;
        for (int c = cf; c < ncyc; ++c) cycle(c, T0{}, T0{});
    } else {
    if (nblk > 0) load(0, cur);
    for (int b = 0; b < nblk; ++b) {
        const int mb = b * SB;
        uint32_t nxt[W];
        if (b + 1 < nblk) load(mb + SB, nxt);
#pragma unroll
        for (int sb = 0; sb < SB / S; ++sb) {
            const int m0 = mb + sb * S;
            if (m0 - LMAX >= a.fuse_lo && m0 + S <= a.fuse_hi) {
                /* Inside the Tukey window's rectangle (weight exactly 1.0) every windowed
                 * sample and lag partner is the integer sample itself, and the product of two
                 * integers below 2^26 is exact in a double: RN(acc + RN(p * a)) ==
                 * fma(p, a, acc).  One fused op per term instead of a multiply and an add,
                 * bit-identical. */
#pragma unroll
                for (int t = 0; t < S; ++t) {
                    const double av = (double)sample(cur, sb * S + t);
                    ring[t] = av;
#pragma unroll
                    for (int l = 0; l <= LMAX; ++l) acc[l] = __builtin_fma(ring[(t - l + S) % S], av, acc[l]);
                }
            } else {
#pragma unroll
                for (int t = 0; t < S; ++t) {
                    const double av = (double)sample(cur, sb * S + t) * win[m0 + t];
                    ring[t] = av;
#pragma unroll
                    for (int l = 0; l <= LMAX; ++l) {
                        const double prev = ring[(t - l + S) % S];
                        acc[l] = acc[l] + prev * av;
                    }
                }
            }
        }
#pragma unroll
        for (int w = 0; w < W; ++w) cur[w] = nxt[w];
    }
    } /* PK == 2 */
    if (a.acf) {
        double* o = a.acf + gid * 33;
#pragma unroll
        for (int l = 0; l < 33; ++l) o[l] = (l <= LMAX && l <= L) ? acc[l < LMAX ? l : LMAX] : 0.0;
    }
    } /* !ACF_IN */

    lpc_finish<LMAX>(acc, a, rec);
}


/* k_lpc_tile: the same per-lane chains (and lpc_finish) for int16 samples at L <= 12, with
 * the samples staged through LDS in whole 128-byte lines: per 64-sample tile each wave
 * copies its 64 rows' lines with eight global_load_lds_dwordx4 (one instruction = 8 rows x
 * 128 B, DMA straight into LDS), each lane then reads its row's 128 B into registers and
 * the wave issues the next tile's copies at once, so they land behind this tile's f64
 * work.  k_lpc's own loads are lane-strided (64 rows per 16-byte instruction: every
 * instruction touches 64 lines, and a line's two halves arrive 32 samples apart, when L2
 * may have dropped it).
 * LDS image of a wave (8 KB): slot 8 r + j (16 B) holds segment (j + r) & 7 of row r, so the
 * lanes reading segment k of their own rows hit 16 distinct 16-byte columns per quarter
 * wave (no bank conflicts); the DMA writes lane-linearly, so the rotation is applied to the
 * per-lane SOURCE address. */
template <int LMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LMAX <= 12 ? 4 : 1))) void k_lpc_tile(LpcArgs a) {
    __shared__ __align__(16) uint4 tiles[4 * 512];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t wave0 = (int64_t)blockIdx.x * 256 + wid * 64;
    if (wave0 >= a.count) return; /* wave-uniform; the host launches whole waves (count % 64 == 0) */
    const int64_t gid = wave0 + lane;
    const int n = a.n, L = a.L;
    int32_t* __restrict__ rec = a.rec + gid * a.rec_words;
    constexpr int S = ((LMAX + 1 + 7) / 8) * 8;
    static_assert(32 % S == 0, "ring length divides a half tile");
    double acc[LMAX + 1];
    if (n >= 4 && n <= 7) { /* tukey: nr == 0 -> pi * 0 / 0 (encoder.py:437) */
        rec[0] = ST_ZERODIV | (FLACMI_SITE_TUKEY << 16);
        rec[1] = 0;
        if (a.acf)
            for (int l = 0; l < 33; ++l) a.acf[gid * 33 + l] = 0.0;
        return;
    }
    double ring[S];
#pragma unroll
    for (int t = 0; t < S; ++t) ring[t] = 0.0;
#pragma unroll
    for (int l = 0; l <= LMAX; ++l) acc[l] = 0.0;
    const int M = n - 1; /* the last sample never enters a product (encoder.py:449) */
    /* the window through the constant address space: scalar loads (a generic pointer read
     * beside the LDS-DMA intrinsic is loaded per lane and waited for with vmcnt(0), which
     * would also wait for the next tile's copies) */
    const __attribute__((address_space(4))) double* win = (const __attribute__((address_space(4))) double*)a.window;
    const int ntile = (M + 63) >> 6;
    uint4* tile = tiles + 512 * wid;
    /* the DMA source of lane l in copy j: row 8 j + l / 8, segment (l % 8 + l / 8) % 8 of the
     * tile, clamped to the row's stride (a clamped segment lies at or past n, whose samples
     * the tile masks) */
    const int seg = ((lane & 7) + (lane >> 3)) & 7;
    const int smax = (int)a.stride - 8;
    const int16_t* row0 = (const int16_t*)a.samples + (a.unit0 + wave0 + (lane >> 3)) * a.stride;
    const int64_t rstep = 8 * a.stride; /* elements from copy j to j + 1 (wave-uniform) */
    auto issue = [&](int m0) __attribute__((always_inline)) {
        int off = m0 + 8 * seg;
        off = off < smax ? off : smax;
        const int16_t* p = row0 + off;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(p + j * rstep),
                                             (void __attribute__((address_space(3)))*)(tile + 64 * j), 16, 0, 0);
    };
    /* this lane's row in the image: segment k at slot 8 lane + ((k - lane) & 7) */
    const uint4* myrow = tile + 8 * lane;
    const int rot = (-lane) & 7;
    using T0 = std::integral_constant<bool, false>;
    using T1 = std::integral_constant<bool, true>;
    /* one 64-sample tile; RECT: the whole tile lies inside the window's rectangle and below M */
    auto tile_body = [&](int tI, auto rectc) __attribute__((always_inline)) {
        constexpr bool RECT = decltype(rectc)::value;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* this wave's copies have landed */
        /* two halves of 32 samples; the next tile's copies go out once the second half is
         * read out of the image (they land behind its f64 work) */
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            /* (a fence per half: hoisted, the 64 window values' scalar loads spill SGPRs) */
            __builtin_amdgcn_sched_barrier(0);
            const int m0 = (tI << 6) + 32 * h;
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 q = myrow[(4 * h + k + rot) & 7];
                v[4 * k] = q.x, v[4 * k + 1] = q.y, v[4 * k + 2] = q.z, v[4 * k + 3] = q.w;
            }
            if (h == 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* read out before the copies overwrite it */
                if (tI + 1 < ntile) issue((tI + 1) << 6);
            }
            if (!RECT && m0 + 32 > M) { /* the last samples: those >= M are zero, as k_lpc loads them */
#pragma unroll
                for (int w = 0; w < 16; ++w) {
                    const int m = m0 + 2 * w;
                    v[w] = m >= M ? 0u : (m + 1 >= M ? (v[w] & 0xffffu) : v[w]);
                }
            }
#pragma unroll
            for (int sb = 0; sb < 32 / S; ++sb) {
                const int ms = m0 + sb * S;
                if constexpr (RECT) {
                    /* inside the Tukey rectangle: exact integer products, one FMA per term (k_lpc) */
#pragma unroll
                    for (int t = 0; t < S; ++t) {
                        const int i = sb * S + t;
                        const double av = (double)((i & 1) ? (int32_t)v[i >> 1] >> 16 : (int32_t)(v[i >> 1] << 16) >> 16);
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) acc[l] = __builtin_fma(ring[(t - l + S) % S], av, acc[l]);
                    }
                } else { /* the reference's multiply and add (exact inside the rectangle too) */
#pragma unroll
                    for (int t = 0; t < S; ++t) {
                        const int i = sb * S + t;
                        const double av =
                            (double)((i & 1) ? (int32_t)v[i >> 1] >> 16 : (int32_t)(v[i >> 1] << 16) >> 16) * win[ms + t];
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) {
                            const double prev = ring[(t - l + S) % S];
                            acc[l] = acc[l] + prev * av;
                        }
                    }
                }
            }
        }
    };
    /* the rectangle's whole tiles [t1, t2) between the two tapers: three loops, one path each
     * (one loop holding both paths needs more registers: 154 VGPRs against 128 here) */
    int t1 = (a.fuse_lo + LMAX + 63) >> 6;
    if (a.fuse_lo + LMAX <= 0) t1 = 0;
    int t2 = min(a.fuse_hi, M) >> 6; /* (tI + 1) * 64 <= min(fuse_hi, M) */
    if (t2 > ntile) t2 = ntile;
    if (t1 > t2) t1 = t2;
    if (ntile > 0) issue(0);
    for (int tI = 0; tI < t1; ++tI) tile_body(tI, T0{});
    for (int tI = t1; tI < t2; ++tI) tile_body(tI, T1{});
    for (int tI = t2; tI < ntile; ++tI) tile_body(tI, T0{});
    if (a.acf) {
        double* o = a.acf + gid * 33;
#pragma unroll
        for (int l = 0; l < 33; ++l) o[l] = (l <= LMAX && l <= L) ? acc[l < LMAX ? l : LMAX] : 0.0;
    }
    lpc_finish<LMAX>(acc, a, rec);
}


/* FLACMI_LPC_TILE=0 selects k_lpc for int16 rows (A/B and parity comparison) */
static bool lpc_tile_enabled() {
    static const bool on = [] {
        const char* e = getenv("FLACMI_LPC_TILE");
        return !(e && e[0] == '0');
    }();
    return on;
}

template <int LMAX>
static hipError_t launch_lpc_T(const LpcArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((a.count + 255) / 256));
    if constexpr (LMAX <= 12) {
        /* whole waves of rows made of whole 16-byte segments (the tile's clamp stays inside
         * the row) through k_lpc_tile; the last count % 64 units through k_lpc */
        const int64_t full = a.count & ~(int64_t)63;
        if (a.sample_bytes == 2 && lpc_tile_enabled() && a.stride % 8 == 0 && a.stride >= 8 && full > 0) {
            LpcArgs t = a;
            t.count = full;
            hipLaunchKernelGGL((k_lpc_tile<LMAX>), dim3((unsigned)((full + 255) / 256)), dim3(256), 0, s, t);
            if (full == a.count) return hipGetLastError();
            LpcArgs r = a;
            r.unit0 += full;
            r.count = a.count - full;
            r.rec += full * a.rec_words;
            if (r.acf) r.acf += full * 33;
            hipLaunchKernelGGL((k_lpc<LMAX, int16_t>), dim3((unsigned)((r.count + 255) / 256)), dim3(256), 0, s, r);
            return hipGetLastError();
        }
    }
    if (a.sample_bytes == 2)
        hipLaunchKernelGGL((k_lpc<LMAX, int16_t>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_lpc<LMAX, int32_t>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_lpc_from_acf(const LpcArgs& a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_lpc<32, int32_t, true>), dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int LMAX>
static const void* lpc_kernel_T(const LpcArgs& a) {
    if constexpr (LMAX <= 12)
        if (a.sample_bytes == 2 && lpc_tile_enabled() && a.stride % 8 == 0 && a.stride >= 8)
            return reinterpret_cast<const void*>(&k_lpc_tile<LMAX>);
    return a.sample_bytes == 2 ? reinterpret_cast<const void*>(&k_lpc<LMAX, int16_t>)
                               : reinterpret_cast<const void*>(&k_lpc<LMAX, int32_t>);
}

int64_t lpc_units_per_round(const LpcArgs& a) {
    const void* f = a.L <= 4 ? lpc_kernel_T<4>(a) : a.L <= 8 ? lpc_kernel_T<8>(a) : a.L <= 12 ? lpc_kernel_T<12>(a)
                  : a.L <= 16 ? lpc_kernel_T<16>(a) : lpc_kernel_T<32>(a);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    /* the occupancy query costs about a millisecond of host time: once per (device, kernel) */
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, int64_t> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, f);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 0, nb = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 256, 0) != hipSuccess)
        return 0;
    return cache[key] = (int64_t)nb * 256 * cus;
}

hipError_t launch_lpc(const LpcArgs& a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    if (a.L <= 4) return launch_lpc_T<4>(a, s);
    if (a.L <= 8) return launch_lpc_T<8>(a, s);
    if (a.L <= 12) return launch_lpc_T<12>(a, s);
    if (a.L <= 16) return launch_lpc_T<16>(a, s);
    return launch_lpc_T<32>(a, s);
}


}  // namespace flacmi
